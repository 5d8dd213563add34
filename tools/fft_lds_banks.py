"""Search an XOR swizzle for the workgroup FFT exchanges (device_fft.hpp: T lanes x E complex,
N = T*E points, 16-B slots, passes of log2(E) stages). Costs model MI355X_MICROARCH.md §LDS per
wave instruction: ds_write_b128 serves 8 groups of 8 contiguous lanes (conflict free iff slot
mod 8 distinct), ds_read_b128 4 groups of 16 lanes (slot mod 16). pad(j) = j ^ f(j), f linear
over GF(2) in bits 3..L-1 of j writing bits 0..3 (bit 3 only from bits >= 4): a bijection.
usage: python tools/fft_lds_banks.py T E L"""
import sys
import numpy as np

T, E, L = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (64, 8, 9)
R = E.bit_length() - 1
NPASS = (L + R - 1) // R
rng = np.random.default_rng(0)
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
W = np.stack([idx(pw, e) for pw, _ in pairs for e in range(E)])
Rd = np.stack([idx(pr, e) for _, pr in pairs for e in range(E)])
NB = L - 3

def f_of(j, M):
    f = np.zeros_like(j)
    for b in range(NB):
        f ^= ((j >> (3 + b)) & 1) * M[b]
    return f

def ndistinct_deficit(vals, groups, size):
    c = 0
    for g in groups:
        blk = np.sort(vals[:, g], axis=1)
        c += int((size - (1 + (np.diff(blk, axis=1) != 0).sum(axis=1))).sum())
    return c

def cost(M):
    return ndistinct_deficit((W ^ f_of(W, M)) & 7, GW, 8) + ndistinct_deficit((Rd ^ f_of(Rd, M)) & 15, GR, 16)

def rand_M():
    return [int(rng.integers(8))] + [int(rng.integers(16)) for _ in range(NB - 1)]

best = (cost([0] * NB), [0] * NB)
print("identity cost", best[0])
for it in range(40000):
    M = rand_M() if it % 4 == 0 else list(best[1])
    if it % 4:
        b = int(rng.integers(NB)); M[b] = int(rng.integers(8 if b == 0 else 16))
    c = cost(M)
    if c < best[0]:
        best = (c, M)
        if c == 0:
            break
print(f"T={T} E={E} L={L}: best extra conflict cycles {best[0]}, masks for bits 3..{L-1}: {best[1]}")
