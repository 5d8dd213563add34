"""Dump the GPU's packed level-1 digits of the first CMUX step and compare with numpy."""
import ctypes as C
import sys
sys.path.insert(0, "tests")
import numpy as np
import product_lib as PL
from product_lib import omr_amd as A

Q1 = 134215681
_, _, dk = PL.keys()
det = A.Detector(dk)
L = A.lib()
L.omr_blind_rotate_level1_mode.restype = C.c_int
L.omr_blind_rotate_level1_mode.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_int]
def br1(la, lb, mode):
    out = np.zeros((1, 2, 1024), np.uint64)
    rc = L.omr_blind_rotate_level1_mode(det._h, la.ctypes.data, lb.ctypes.data, C.c_size_t(1),
                                        out.ctypes.data, C.c_int(mode))
    assert rc == 0
    return out[0]
def centre(x): x = x.astype(np.int64); return np.where(x > Q1 // 2, x - Q1, x)
def rot(p, r):
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
lb = np.array([37], np.uint16)
acc = centre(br1(np.zeros(512, np.uint16), lb, 1))
for a in (77, 1000):
    la = np.zeros(512, np.uint16); la[0] = a
    pk = br1(la, lb, 2).astype(np.uint32)
    for p in range(2):
        v = rot(acc[p], a) - acc[p]
        vc = np.where(v > Q1 // 2, v - Q1, np.where(v < -(Q1 // 2), v + Q1, v))
        want = digits(vc)
        got = [((pk[p] >> (8 * k)) & 0xff).astype(np.int8).astype(np.int64) for k in range(4)]
        for k in range(4):
            bad = np.flatnonzero(got[k] != want[k])
            print(f"a={a} p={p} k={k}: bad {bad.size} idx {bad[:4]} got {got[k][bad[:4]]} want {want[k][bad[:4]]} "
                  f"v {vc[bad[:4]]} acc {acc[p][bad[:4]]}")

# the same digit polys through the standalone FFT product
for a in (1000,):
    for p in range(2):
        v = rot(acc[p], a) - acc[p]
        vc = np.where(v > Q1 // 2, v - Q1, np.where(v < -(Q1 // 2), v + Q1, v))
        for k, d in enumerate(digits(vc)):
            one = np.zeros(1024, np.uint32); one[0] = 1
            g = centre(det.fft1_mul((d % Q1).astype(np.uint32)[None], one[None])[0])
            bad = np.flatnonzero(g != d)
            print(f"fft1_mul a={a} p={p} k={k} (key=1): bad {bad.size} idx {bad[:4]} got {g[bad[:4]]} want {d[bad[:4]]}")
