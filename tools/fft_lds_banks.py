"""Search an XOR swizzle for the 512-point wave FFT exchange (64 lanes x 8 complex, 16-B slots).
Costs model MI355X_MICROARCH.md §LDS: ds_write_b128 serves 8 groups of 8 contiguous lanes
(conflict free iff slot mod 8 distinct), ds_read_b128 serves 4 groups of 16 lanes (slot mod 16).
pad(j) = j ^ f(j), f linear over GF(2) in bits 3..8 of j, writing bits 0..3 (bit 3 only from
bits 4..8), so pad is a bijection on [0, 512)."""
import numpy as np

rng = np.random.default_rng(0)
tid = np.arange(64)
def idx(p, e):
    if p == 0: return e * 64 + tid
    if p == 1: return ((tid >> 3) << 6) | (e << 3) | (tid & 7)
    return (tid << 3) | e
G = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
     list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G += [[x + 32 for x in g] for g in G]
pairs = [(0, 1), (1, 2), (2, 1), (1, 0)]
W = np.stack([idx(pw, e) for pw, _ in pairs for e in range(8)])   # [32][64] write indices
R = np.stack([idx(pr, e) for _, pr in pairs for e in range(8)])   # [32][64] read indices
def f_of(j, M):
    f = np.zeros_like(j)
    for b in range(6):
        f ^= ((j >> (3 + b)) & 1) * M[b]
    return f
def cost(M):
    w = (W ^ f_of(W, M)) & 7
    r = (R ^ f_of(R, M)) & 15
    c = 0
    for g in range(8):
        blk = np.sort(w[:, 8 * g:8 * g + 8], axis=1)
        c += int((8 - (1 + (np.diff(blk, axis=1) != 0).sum(axis=1))).sum())
    for g in G:
        blk = np.sort(r[:, g], axis=1)
        c += int((16 - (1 + (np.diff(blk, axis=1) != 0).sum(axis=1))).sum())
    return c
def rand_M():
    return [int(rng.integers(8))] + [int(rng.integers(16)) for _ in range(5)]
best = (cost([0] * 6), [0] * 6)
for it in range(20000):
    M = rand_M() if it % 4 == 0 else list(best[1])
    if it % 4:
        b = int(rng.integers(6)); M[b] = int(rng.integers(8 if b == 0 else 16))
    c = cost(M)
    if c < best[0]:
        best = (c, M)
        print(it, c, M, flush=True)
        if c == 0:
            break
print("best extra conflict cycles:", best[0], "rows (bits 3..8 of j -> xor mask):", best[1])
