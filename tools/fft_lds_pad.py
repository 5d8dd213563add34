"""Search an ADDITIVE padding pad(j) = j + sum_k (j >> s_k) for the wave/workgroup FFT exchanges
(16-B slots). Because the lane and element fields of an exchange index are disjoint bit ranges,
pad(lanepart | epart) = pad(lanepart) + pad(epart): every access is one per-lane base register
plus an immediate offset (no per-element address registers). Bank model as tools/fft_lds_banks.py.
usage: python tools/fft_lds_pad.py T E L"""
import itertools
import sys
import numpy as np

T, E, L = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (64, 8, 9)
R = E.bit_length() - 1
NPASS = (L + R - 1) // R
tid = np.arange(T)

def idx(p, e):
    s0 = p * R
    r = min(R, L - s0)
    lb = L - s0 - r
    F = (tid << (R - r)) | (e >> r)
    ep = e & ((1 << r) - 1)
    return ((F >> lb) << (L - s0)) | (ep << lb) | (F & ((1 << lb) - 1))

G16 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
       list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G16 += [[x + 32 for x in g] for g in G16]
GR = [[w * 64 + x for x in g] for w in range(T // 64) for g in G16]
GW = [list(range(8 * g, 8 * g + 8)) for g in range(T // 8)]
pairs = [(p, p + 1) for p in range(NPASS - 1)] + [(p + 1, p) for p in range(NPASS - 1)]

def deficit(vals, groups, size):
    c = 0
    for g in groups:
        c += size - len(set(vals[g].tolist()))
    return c

def cost(shifts):
    pad = lambda j: j + sum((j >> s) for s in shifts)
    c = 0
    for pw, pr in pairs:
        for e in range(E):
            c += deficit(pad(idx(pw, e)) & 7, GW, 8) + deficit(pad(idx(pr, e)) & 15, GR, 16)
    return c

best = None
for n in (1, 2, 3):
    for sh in itertools.combinations(range(2, L), n):
        c = cost(sh)
        extra = sum((1 << L) >> s for s in sh)
        if best is None or (c, extra) < best[0]:
            best = ((c, extra), sh)
print(f"T={T} E={E} L={L}: best additive pad shifts {best[1]}: extra conflict cycles {best[0][0]}, "
      f"buffer {(1 << L) + best[0][1]} slots")
