"""Split inverse of the two-CU latency kernel (br2x_kernel, device_ntt.hpp HalfInv), restated
with exact integers: after the MAC each 256-thread group holds partial sums for all 2048 NTT
positions in CmuxNtt's P3 layout (thread t, register e at cmux_idx(3, t, e)). Inverse stage 10
(index bit 0, register bit 1 of e) is applied by each group to its own partials; then group g keeps
the 4 registers with e bit 1 == g -- the positions with index bit 0 == g, which stages 9..0 never
combine with the other half -- and runs stages 9..0 of that 1024-point half on 256 threads x 4
registers f through layouts Q0 -> Q4 (two permlane relayouts, one wave-local and one cross-wave
LDS exchange). Q4 puts coefficient 2 t + g + 512 f on thread t, register f. The model checks that
this equals the full unscaled inverse (N * a), and that the twiddle reads of the stages hit the
same table entries as the plain tree (stage 9 through the permuted tw2c slot of CmuxNtt)."""
import numpy as np

import oracle_lib as O
from test_cmux_layout import Q2, N, T, cmux_idx, cmux_tw_off, twiddles

F = 4
TID = np.arange(T)


def bit(v, b):
    return (v >> b) & 1


def jq(p, g, t, f):
    """Index j (bit 0 = g) held by register f of thread t of group g in half layout Q<p>."""
    f0, f1 = bit(f, 0), bit(f, 1)
    t_ = [bit(t, k) for k in range(8)]
    if p == 0:    # = P3 restricted to e bit 1 == g: f0 = e bit 0 (j2), f1 = e bit 2 (j1)
        jb = {1: f1, 2: f0, 3: t_[4], 4: t_[5], 5: t_[0], 6: t_[1], 7: t_[2], 8: t_[3], 9: t_[6], 10: t_[7]}
    elif p == 1:  # permlanes: f0 <-> lane bit 4, f1 <-> lane bit 5
        jb = {1: t_[5], 2: t_[4], 3: f0, 4: f1, 5: t_[0], 6: t_[1], 7: t_[2], 8: t_[3], 9: t_[6], 10: t_[7]}
    elif p == 2:  # wave-local LDS exchange
        jb = {5: f0, 6: f1, 7: t_[4], 8: t_[5], 1: t_[3], 2: t_[2], 3: t_[1], 4: t_[0], 9: t_[6], 10: t_[7]}
    elif p == 3:  # permlanes again
        jb = {7: f0, 8: f1, 5: t_[4], 6: t_[5], 1: t_[3], 2: t_[2], 3: t_[1], 4: t_[0], 9: t_[6], 10: t_[7]}
    else:         # cross-wave LDS exchange: coefficient 2 t + g + 512 f
        jb = {9: f0, 10: f1, 1: t_[0], 2: t_[1], 3: t_[2], 4: t_[3], 5: t_[4], 6: t_[5], 7: t_[6], 8: t_[7]}
    return g | sum(v << b for b, v in jb.items())


def e_of(g, f):  # P3 register of half register f (Q0)
    return (f & 1) | (g << 1) | (((f >> 1) & 1) << 2)


def test_half_layouts_bijective_and_local():
    for g in (0, 1):
        for p in range(5):
            idx = sorted(jq(p, g, t, f) for t in range(T) for f in range(F))
            assert idx == list(range(g, N, 2))
        for t in range(T):
            for f in range(F):
                assert jq(0, g, t, f) == cmux_idx(3, t, e_of(g, f))
                # wave bits (index bits 10, 9) stay on the wave until the cross-wave exchange
                for p in range(4):
                    assert jq(p, g, t, f) >> 9 == t >> 6
                assert jq(4, g, t, f) == 2 * t + g + 512 * f


def test_permlane_relayouts():
    # swap_lane_bit<4>(x[f], x[f | 1]) and swap_lane_bit<5>(x[f], x[f | 2]): register bit 0 <-> lane
    # bit 4, register bit 1 <-> lane bit 5 (CmuxNtt::swap23's primitive)
    for g in (0, 1):
        for pf, pt in ((0, 1), (2, 3)):
            for t in range(T):
                for f in range(F):
                    src_t = (t & ~0x30) | (bit(f, 0) << 4) | (bit(f, 1) << 5)
                    src_f = bit(t, 4) | (bit(t, 5) << 1)
                    assert jq(pf, g, src_t, src_f) == jq(pt, g, t, f)


# stage s of the inverse pairs index bit 10 - s; the register bit holding it per layout
STAGES = {0: (9, 8), 1: (7, 6), 2: (5, 4), 3: (3, 2), 4: (1, 0)}


def rbit_q(p, s):
    b = 10 - s
    f = [x for x in (1, 2) if jq(p, 0, 0, x) & (1 << b)]
    assert len(f) == 1 and f[0] in (1, 2)
    return f[0]


def model_split_inverse(X, tw, tw2c):
    """X: NTT-domain values (index j). Returns the coefficient values per (g, t, f) in Q4."""
    # stage 10 on the P3 layout (both halves still together; each group does this on its partials)
    x = {(t, e): X[cmux_idx(3, t, e)] for t in range(T) for e in range(8)}
    for t in range(T):
        for e in range(8):
            if e & 2:
                continue
            w = tw2c[(2 << 10) - 1 - cmux_tw_off(3, 10, t, e)]
            u, v = x[(t, e)], x[(t, e + 2)]
            x[(t, e)], x[(t, e + 2)] = (u + v) % Q2, (v - u) * w % Q2
    out = {}
    for g in (0, 1):
        h = {(t, f): x[(t, e_of(g, f))] for t in range(T) for f in range(F)}
        for p in range(5):
            if p:
                by = {jq(p - 1, g, t, f): h[(t, f)] for t in range(T) for f in range(F)}
                h = {(t, f): by[jq(p, g, t, f)] for t in range(T) for f in range(F)}
            for s in STAGES[p]:
                hb = rbit_q(p, s)
                for t in range(T):
                    for f in range(F):
                        if f & hb:
                            continue
                        node = jq(p, g, t, f) >> (11 - s)
                        if s == 9:  # the permuted CmuxNtt slot (Q0 is P3 restricted)
                            wv = tw2c[(2 << 9) - 1 - cmux_tw_off(3, 9, t, e_of(g, f))]
                            assert wv == tw[(2 << 9) - 1 - node]
                        else:
                            wv = tw[(2 << s) - 1 - node]
                            assert s > 8 or wv == tw2c[(2 << s) - 1 - node]
                        u, v = h[(t, f)], h[(t, f + hb)]
                        h[(t, f)], h[(t, f + hb)] = (u + v) % Q2, (v - u) * wv % Q2
        for t in range(T):
            for f in range(F):
                out[(g, t, f)] = h[(t, f)]
    return out


def test_split_inverse_equals_full_inverse():
    rng = np.random.default_rng(21)
    a = rng.integers(0, Q2, N, dtype=np.uint64)
    X = [int(v) for v in O.ntt(2, a.copy())]
    tw, tw2c = twiddles()
    out = model_split_inverse(X, tw, tw2c)
    for (g, t, f), v in out.items():
        assert v == (N * int(a[2 * t + g + 512 * f])) % Q2
