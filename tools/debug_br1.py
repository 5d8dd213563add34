"""GPU debug checks of the level-1 path: FFT product vs exact negacyclic product, and blind
rotations with 0 / 1 / 2 CMUX steps vs the oracle."""
import sys
sys.path.insert(0, "tests")
import numpy as np
import product_lib as PL
from product_lib import omr_amd as A
import oracle_lib as O

Q1 = 134215681
import os; print("lib:", os.environ.get("OMR_GPU_LIB", "default"))
a_sk, _, dk = PL.keys()
det = A.Detector(dk)
rng = np.random.default_rng(3)
n = 4
a = rng.integers(-17, 18, (n, 1024))
k = rng.integers(0, Q1, (n, 1024))
def negacyc(x, y):
    full = np.convolve(x.astype(object), y.astype(object))
    r = full[:1024].copy(); r[:1023] -= full[1024:]
    return np.array([int(v) % Q1 for v in r], dtype=np.uint64)
got = det.fft1_mul((a % Q1).astype(np.uint32), k.astype(np.uint32))
for i in range(n):
    ref = negacyc(a[i], np.where(k[i] > Q1 // 2, k[i] - Q1, k[i]))
    print("fft1_mul", i, "match" if np.array_equal(got[i], ref) else f"MISMATCH {np.sum(got[i] != ref)} coeffs, first {got[i][:4]} vs {ref[:4]}")
orc = O.OracleDetector(dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key)
for case, la_nz in [("0 steps", {}), ("1 step", {0: 5}), ("1 step a=1000", {3: 1000}), ("2 steps", {0: 5, 7: 77})]:
    la = np.zeros(512, np.uint16)
    for i, v in la_nz.items(): la[i] = v
    lb = np.array([37], np.uint16)
    g = det.blind_rotate_level1(la[None], lb)[0]
    r = orc.br1(la, 37)
    ok = np.array_equal(g, r)
    print(case, "match" if ok else f"MISMATCH mask {np.sum(g[0] != r[0])} body {np.sum(g[1] != r[1])}; g {g[0][:3]} r {r[0][:3]}")

# exact single CMUX step in numpy from the 0-step accumulator
def centre(x): x = x.astype(np.int64); return np.where(x > Q1 // 2, x - Q1, x)
def rot(p, r):  # X^r * p
    out = np.zeros(1024, np.int64)
    for j in range(1024):
        t = j - r; s = 1
        if t < 0: t += 1024; s = -1
        if t < 0: t += 1024; s = 1
        out[j] = s * p[t]
    return out
def digits(v):
    y = (v + 64) >> 7; ds = []
    for k in range(3):
        c = (y + 16) >> 5; ds.append(y - (c << 5)); y = c
    ds.append(y); return ds
def nc(x, y):
    full = np.convolve(x, y); r = full[:1024].copy(); r[:1023] -= full[1024:]; return r
bsk1 = np.asarray(dk.bsk1, dtype=np.uint32).reshape(512, 8, 2, 1024)
la0 = np.zeros(512, np.uint16)
acc = centre(det.blind_rotate_level1(la0[None], np.array([37], np.uint16))[0])
for (i, a) in [(0, 1000), (3, 5), (3, 1000), (0, 77), (7, 77)]:
    out = acc.copy()
    for p in range(2):
        v = rot(acc[p], a) - acc[p]
        v = np.where(v > Q1 // 2, v - Q1, np.where(v < -(Q1 // 2), v + Q1, v))
        for k, d in enumerate(digits(v)):
            for o in range(2):
                out[o] += nc(d, centre(bsk1[i, p * 4 + k, o]))
    exp = (out % Q1).astype(np.uint64)
    la = np.zeros(512, np.uint16); la[i] = a
    g = det.blind_rotate_level1(la[None], np.array([37], np.uint16))[0]
    r = orc.br1(la, 37)
    diff = (g.astype(np.int64) - exp.astype(np.int64)) % Q1
    diff = np.where(diff > Q1 // 2, diff - Q1, diff)
    print(f"i={i} a={a}: gpu==exact {np.array_equal(g, exp)} oracle==exact {np.array_equal(r, exp)} "
          f"nz diffs mask {np.count_nonzero(diff[0])} body {np.count_nonzero(diff[1])} "
          f"max|diff| {np.abs(diff).max()} first nz idx {np.flatnonzero(diff[0])[:6]}")

# digit probe: BSK1 with only row r of step 0, component A, equal to the constant 1
import dataclasses
for a_rot in (77, 1000):
    for r in range(8):
        b1 = np.zeros_like(bsk1); b1[0, r, 0, 0] = 1
        dkr = A.DetectionKey(bsk1=b1, ksk=dk.ksk, bsk2=dk.bsk2, trace_key=dk.trace_key)
        d2 = A.Detector(dkr)
        la = np.zeros(512, np.uint16); la[0] = a_rot
        g = centre(d2.blind_rotate_level1(la[None], np.array([37], np.uint16))[0])
        p, k = divmod(r, 4)
        v = rot(acc[p], a_rot) - acc[p]
        v = np.where(v > Q1 // 2, v - Q1, np.where(v < -(Q1 // 2), v + Q1, v))
        d = digits(v)[k]
        bad = np.flatnonzero(g[0] != d)
        print(f"a={a_rot} row {r}: digit poly {'OK' if bad.size == 0 else 'BAD'} n_bad={bad.size} "
              f"idx {bad[:5]} got {g[0][bad[:5]]} want {d[bad[:5]]}")
        d2.close()
