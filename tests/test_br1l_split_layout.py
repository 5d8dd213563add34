"""Split level-1 inverse of the latency kernel (br1l_kernel with OMR_BR1L_SPLIT, latency_kernels.hpp
HalfInv1), restated in numpy: the MAC leaves output o's spectrum in LDS in WgFft's P3 order
(register e of lane l at index jidx(3, l, e)). Two waves per output read all of it, apply inverse
stage 8 (index bit 0, WgFft::inv2) redundantly, and wave g keeps the 4 registers with index bit
0 == g -- a 256-point half that stages 7..0 never mix with the other -- and finishes it alone:
radix-4 inverse passes (stages 7/6, 5/4, 3/2, 1/0) on layouts H0 -> H3 (a wave-local LDS exchange,
a permlane relayout, another wave-local exchange). H3 puts point g + 2 l + 128 f on lane l,
register f. Checked against tools/fft_exactness.py's model of the one-wave inverse."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import fft_exactness as FX  # noqa: E402

n, L = 512, 9
LANE = np.arange(64)


def bit(v, b):
    return (v >> b) & 1


def jh(p, g, l, f):
    """Index (bit 0 = g) of register f on lane l in half layout H<p> (HalfInv1::jh)."""
    f0, f1 = bit(f, 0), bit(f, 1)
    lb = [bit(l, k) for k in range(6)]
    if p == 0:    # P3 restricted to e bit 2 == g: f = e & 3 (f0 = j1, f1 = j2), lane & 31 -> j8..j4, l5 -> j3
        jb = {1: f0, 2: f1, 3: lb[5], 4: lb[0], 5: lb[1], 6: lb[2], 7: lb[3], 8: lb[4]}
    elif p == 1:  # wave-local exchange
        jb = {3: f0, 4: f1, 5: lb[4], 6: lb[5], 1: lb[0], 2: lb[1], 7: lb[2], 8: lb[3]}
    elif p == 2:  # permlanes: f0 <-> lane bit 4, f1 <-> lane bit 5
        jb = {5: f0, 6: f1, 3: lb[4], 4: lb[5], 1: lb[0], 2: lb[1], 7: lb[2], 8: lb[3]}
    else:         # wave-local exchange: point g + 2 l + 128 f
        jb = {7: f0, 8: f1, 1: lb[0], 2: lb[1], 3: lb[2], 4: lb[3], 5: lb[4], 6: lb[5]}
    return g | sum(v << b for b, v in jb.items())


def jidx3(l, e):
    return ((l & 31) << 4) | (bit(l, 5) << 3) | (bit(e, 1) << 2) | (bit(e, 0) << 1) | bit(e, 2)


def tree_half():
    half, eps = [], [n]
    for s in range(L):
        half.append([e // 2 for e in eps])
        eps = [y for e in eps for y in ((e // 2) % (4 * n), (e // 2 + 2 * n) % (4 * n))]
    return half


HALF = tree_half()


def W(s, i):
    return np.exp(1j * np.pi * (HALF[s][i] % (8 * n)) / (2 * n))


# host table of the radix-4 passes (context.hip fft1_half_twiddles): pass stage s in {6, 4, 2, 0},
# block hi < 2^s: (B, A, AB) with A = W(s, hi), B = W(s + 1, 2 hi), at OFF[s] + 3 hi
OFF = {6: 0, 4: 192, 2: 240, 0: 252}


def test_layouts_are_bijections_and_permlane_step():
    for g in (0, 1):
        for p in range(4):
            idx = sorted(jh(p, g, l, f) for l in range(64) for f in range(4))
            assert idx == list(range(g, n, 2))
        for l in range(64):
            for f in range(4):
                assert jh(0, g, l, f) == jidx3(l, f | (g << 2))
                src_l = (l & ~0x30) | (bit(f, 0) << 4) | (bit(f, 1) << 5)
                src_f = bit(l, 4) | (bit(l, 5) << 1)
                assert jh(1, g, src_l, src_f) == jh(2, g, l, f)
                assert jh(3, g, l, f) == g + 2 * l + 128 * f


def inv_pass(x, p, s, g):
    """Inverse radix-4 block (stages s + 1, s) on layout H<p>: inet4, then x * conj(1, B, A, AB).
    Registers e = 2 b_hi + b_lo with b_hi = index bit 8 - s, b_lo = bit 7 - s."""
    out = np.empty_like(x)
    for l in range(64):
        j0 = jh(p, g, l, 0)
        hi = j0 >> (L - s)
        A, B = W(s, hi), W(s + 1, 2 * hi)
        o = x[l]
        a0, a1 = o[0] + o[1], o[0] - o[1]
        b0, b1 = o[2] + o[3], -1j * (o[2] - o[3])
        y = np.array([a0 + b0, a1 + b1, a0 - b0, a1 - b1])
        out[l] = y * np.conj(np.array([1, B, A, A * B]))
    return out


def relayout(x, g, pf, pt):
    by = {jh(pf, g, l, f): x[l, f] for l in range(64) for f in range(4)}
    return np.array([[by[jh(pt, g, l, f)] for f in range(4)] for l in range(64)])


def test_split_inverse_equals_one_wave_inverse():
    rng = np.random.default_rng(3)
    X = rng.normal(size=n) + 1j * rng.normal(size=n)   # spectrum by index j
    want = FX.Fft8P().inv(X)                            # one-wave inverse, natural order, x512
    # stage 8 (index bit 0) on all points: pairs (j, j + 1), node j >> 1
    y = X.copy()
    for j in range(0, n, 2):
        w = W(8, j >> 1)
        u, v = y[j], y[j + 1]
        y[j], y[j + 1] = u + v, (u - v) * np.conj(w)
    got = np.zeros(n, dtype=complex)
    for g in (0, 1):
        x = np.array([[y[jh(0, g, l, f)] for f in range(4)] for l in range(64)])
        for p, s in ((0, 6), (1, 4), (2, 2), (3, 0)):
            if p:
                x = relayout(x, g, p - 1, p)
            # b_hi / b_lo of this pass are register bits 1 / 0 in H<p>
            assert all(bit(jh(p, g, 0, f), 8 - s) == bit(f, 1) and bit(jh(p, g, 0, f), 7 - s) == bit(f, 0)
                       for f in range(4))
            x = inv_pass(x, p, s, g)
        for l in range(64):
            for f in range(4):
                got[jh(3, g, l, f)] = x[l, f]
    assert np.max(np.abs(got - want)) < 1e-9 * np.max(np.abs(want))
