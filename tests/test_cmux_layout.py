"""Level-2 CMUX transform layout (tfhe-omr_amd/csrc/device_ntt.hpp, CmuxNtt / cmux_idx /
cmux_tw_off / padw, restated here): every pass layout is a bijection, passes 1-3 stay inside one
wave, the permlane swaps of register bits 2, 1 with lane bits 5, 4 turn pass 2 into pass 3, the
W-buffer swizzle is bank-conflict free for both directions of the wave-local exchange, the
permuted stage-9/10 twiddle table is mirror-compatible, and an exact-integer model of the
transform with these layouts equals the oracle NTT at index cmux_idx(3, tid, e) (and its
inverse returns N * a)."""
import numpy as np
import pytest

import oracle_lib as O

Q2 = 1125899906826241
N, T, E = 2048, 256, 8
TID = np.arange(T)


def cmux_idx(p, t, e):
    if p == 0:
        return (e << 8) | t
    if p == 1:
        return ((t >> 5) << 8) | (e << 5) | (t & 31)
    if p == 2:
        return ((t >> 6) << 9) | ((t & 15) << 5) | (e << 2) | (((t >> 5) & 1) << 1) | ((t >> 4) & 1)
    return (((t >> 6) << 9) | ((t & 15) << 5) | (((t >> 5) & 1) << 4) | (((t >> 4) & 1) << 3)
            | ((e & 1) << 2) | (((e >> 2) & 1) << 1) | ((e >> 1) & 1))


def cmux_tw_off(p, s, t, e):
    if s == 9:
        return (e & 1) * 256 + t
    if s == 10:
        return ((((e >> 2) & 1) << 1) | (e & 1)) * 256 + t
    return cmux_idx(p, t, e) >> (11 - s)


def rbit(p, b):
    return b - 8 if p == 0 else b - 5 if p == 1 else b - 2 if p == 2 else (2 if b == 1 else 1)


def padw(j):
    return j ^ (((j >> 5) & 15) << 1) ^ ((j >> 8) & 1)


def brv(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2)


def twiddles():
    g = 22  # smallest primitive root of q2 (oracle/omr_oracle.h)
    psi = pow(g, (Q2 - 1) // (2 * N), Q2)
    tw = [pow(psi, brv(k, 11), Q2) for k in range(N)]
    tw2c = list(tw)
    for s in (9, 10):
        for t in range(T):
            for e in range(E):
                if not e & (4 if s == 9 else 2):
                    tw2c[(1 << s) + cmux_tw_off(3, s, t, e)] = tw[(1 << s) + (cmux_idx(3, t, e) >> (11 - s))]
    return tw, tw2c


def test_layouts_bijective_and_wave_local():
    for p in range(4):
        idx = np.concatenate([cmux_idx(p, TID, e) for e in range(E)])
        assert np.array_equal(np.sort(idx), np.arange(N))
    for p in (1, 2, 3):  # wave bits (tid 7, 6) hold index bits 10, 9 from pass 1 on
        for e in range(E):
            assert np.array_equal(cmux_idx(p, TID, e) >> 9, TID >> 6)


def test_permlane_swap_gives_pass3():
    # v_permlane32_swap(a = x[e], b = x[e | 4]): lanes 32..63 of a <-> lanes 0..31 of b, i.e. register
    # bit 2 <-> lane bit 5; v_permlane16_swap on (x[e], x[e | 2]): register bit 1 <-> lane bit 4
    for t in range(T):
        for e in range(E):
            src_t = (t & ~0x30) | (((e >> 2) & 1) << 5) | (((e >> 1) & 1) << 4)
            src_e = (e & 1) | (((t >> 4) & 1) << 1) | (((t >> 5) & 1) << 2)
            assert cmux_idx(2, src_t, src_e) == cmux_idx(3, t, e)


def test_w_swizzle_conflict_free():
    assert np.array_equal(np.sort(padw(np.arange(N))), np.arange(N))
    # MI355X_MICROARCH.md LDS table: ds_write_b64 serves 16-lane groups (slot mod 16 distinct),
    # ds_read_b64 32-lane groups (slot mod 32 distinct)
    for p in (1, 2):
        for e in range(E):
            s = padw(cmux_idx(p, TID, e))
            for g in range(0, T, 16):
                assert len(set((s[g:g + 16] % 16).tolist())) == 16
            for g in range(0, T, 32):
                assert len(set((s[g:g + 32] % 32).tolist())) == 32
    for e in range(E):  # the wave only touches its own slots (bits 10, 9 = wave)
        assert np.array_equal(padw(cmux_idx(2, TID, e)) >> 9, TID >> 6)


def test_stage9_10_table_mirror():
    tw, tw2c = twiddles()
    for s in (9, 10):
        for t in (0, 77, 255):
            for e in range(E):
                if e & (4 if s == 9 else 2):
                    continue
                off = cmux_tw_off(3, s, t, e)
                node = cmux_idx(3, t, e) >> (11 - s)
                # the kernel's inverse reads tw2c[(2 << s) - 1 - off] for psi^-brv(2^s + node)
                assert tw2c[(2 << s) - 1 - off] == tw[(2 << s) - 1 - node]
                assert tw2c[(1 << s) + off] == tw[(1 << s) + node]


def model_forward(a, tw2c):
    x = {(t, e): int(a[cmux_idx(0, t, e)]) for t in range(T) for e in range(E)}

    def stages(p, s0, s1):
        for s in range(s0, s1):
            h = 1 << rbit(p, 10 - s)
            for t in range(T):
                for e in range(E):
                    if e & h:
                        continue
                    w = tw2c[(1 << s) + cmux_tw_off(p, s, t, e)]
                    u, v = x[(t, e)], x[(t, e + h)] * w % Q2
                    x[(t, e)], x[(t, e + h)] = (u + v) % Q2, (u - v) % Q2

    def relayout(pf, pt):
        by = {cmux_idx(pf, t, e): x[(t, e)] for t in range(T) for e in range(E)}
        for t in range(T):
            for e in range(E):
                x[(t, e)] = by[cmux_idx(pt, t, e)]

    stages(0, 0, 3)
    relayout(0, 1)
    stages(1, 3, 6)
    relayout(1, 2)
    stages(2, 6, 9)
    relayout(2, 3)  # the permlane swaps (test_permlane_swap_gives_pass3)
    stages(3, 9, 11)
    return x


def model_inverse(x, tw2c):
    x = dict(x)

    def stages(p, s0, s1):
        for s in range(s1 - 1, s0 - 1, -1):
            h = 1 << rbit(p, 10 - s)
            for t in range(T):
                for e in range(E):
                    if e & h:
                        continue
                    w = tw2c[(2 << s) - 1 - cmux_tw_off(p, s, t, e)]
                    u, v = x[(t, e)], x[(t, e + h)]
                    x[(t, e)], x[(t, e + h)] = (u + v) % Q2, (v - u) * w % Q2

    def relayout(pf, pt):
        by = {cmux_idx(pf, t, e): x[(t, e)] for t in range(T) for e in range(E)}
        for t in range(T):
            for e in range(E):
                x[(t, e)] = by[cmux_idx(pt, t, e)]

    stages(3, 9, 11)
    relayout(3, 2)
    stages(2, 6, 9)
    relayout(2, 1)
    stages(1, 3, 6)
    relayout(1, 0)
    stages(0, 0, 3)
    return np.array([x[(t, e)] for e in range(E) for t in range(T)], dtype=object)  # index e*256 + t


@pytest.mark.timeout(300)
def test_model_matches_oracle_ntt():
    rng = np.random.default_rng(11)
    a = rng.integers(0, Q2, N, dtype=np.uint64)
    _, tw2c = twiddles()
    x = model_forward(a, tw2c)
    ref = O.ntt(2, a.copy())
    for t in range(T):
        for e in range(E):
            assert x[(t, e)] == int(ref[cmux_idx(3, t, e)])
    back = model_inverse(x, tw2c)
    assert all(int(back[j]) == (N * int(a[j])) % Q2 for j in range(N))
