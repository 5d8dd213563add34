"""The level-2 exact-FFT kernel's transform (tfhe-omr_amd/csrc/br2_fft.hpp, Fft1024) restated in
numpy (tests/fft2_model.py): layouts, permlane relayouts, LDS exchanges and twiddle tree must give
the exact negacyclic product after rounding, with margin, for the external product's worst case
(12 GGSW rows of 2048 digits |d| <= 64 against 25-bit key limbs |k| <= 2^24); every LDS exchange
and the rotation staging must be bank-conflict free under the MI355X lane-group rules."""
import numpy as np
import pytest

import fft2_model as M


def test_layouts_are_bijections_and_relayouts_match():
    for p in M.IDX:
        assert sorted(M.IDX[p].ravel().tolist()) == list(range(M.n))
    assert np.array_equal(M.relayout_perm(M.IDX[0].copy()), M.IDX[1])
    assert np.array_equal(M.relayout_perm(M.IDX[2].copy()), M.IDX[3])
    # exchanges: X moves the wave bits, W keeps each wave's points inside the wave
    assert not np.array_equal(M.IDX[1] >> 4 & 3, M.IDX[2] >> 4 & 3)
    for t in range(M.T):
        assert {M.idx(3, t, e) >> 6 & 3 for e in range(M.E)} == {M.idx(4, t, e) >> 6 & 3 for e in range(M.E)}


@pytest.mark.parametrize("name", sorted(M.SWIZZLES))
def test_exchanges_conflict_free(name):
    sw = M.SWIZZLES[name]
    assert sorted(sw(j) for j in range(M.n)) == list(range(M.n))
    assert M.exchange_cycles(name) == (8.0, 4.0)


def test_rotation_staging_conflict_free():
    w = r = 0
    for wave in range(4):
        for e in range(M.E):
            for h in (0, M.n):
                cs = [M.idx(0, wave * 64 + l, e) + h for l in range(64)]
                w = max(w, M.lds_cycles([M.slot_stage(c) * 8 for c in cs], M.WRITE_B64, 32, 8))
                for a in (1, 63, 64, 65, 1000, 2047, 2048, 4095):
                    rs = [((c - a) % 4096) % 2048 for c in cs]
                    r = max(r, M.lds_cycles([M.slot_stage(x) * 8 for x in rs], M.READ_B64, 64, 8))
    assert (w, r) == (4, 2)


def test_twiddle_table_layout():
    tab = M.twiddle_table()
    assert len(tab) == 1020 and np.allclose(np.abs(tab), 1.0)
    for p in range(1, 5):  # each thread finds its block's twiddles
        for t in range(M.T):
            got = [tab[M.tw_addr(p, t, k)] for k in range(3)]
            assert np.allclose(got, M.block_tw(p, M.tw_index(p, t)))


def test_twiddle_read_cycles():
    """ds_read_b128 twiddle reads: the host (block-major) order has 4-way conflicts (16 cycles per
    wave instruction) in passes 3 and 4; the LDS slots of Fft1024::tw_slot (each twiddle of passes
    3 and 4 in its own array, the block XOR-swizzled) are conflict-free (4) in every pass. (With
    the point-major key layout a permuted table measured 11 % slower, the workgroups drifting apart
    in CMUX step; with the register-major keys this one is 0.8 % faster) The
    slots are a permutation of the table."""
    host, lds = {}, {}
    for p in range(1, 5):
        host[p] = max(M.lds_cycles([M.tw_addr(p, w * 64 + l, k) * 16 for l in range(64)], M.READ_B128, 64, 16)
                      for w in range(4) for k in range(3))
        lds[p] = max(M.lds_cycles([M.tw_lds(p, w * 64 + l, k) * 16 for l in range(64)], M.READ_B128, 64, 16)
                     for w in range(4) for k in range(3))
    assert host == {1: 4, 2: 4, 3: 16, 4: 16}
    assert lds == {1: 4, 2: 4, 3: 4, 4: 4}
    slots = sorted(M.tw_slot(p, b, k) for p in range(1, 5) for b in range(4 ** p) for k in range(3))
    assert slots == list(range(M.TW_LEN))
    # pass-0 constants of the device code: B = e^{i pi/8}, A = e^{i pi/4}, AB = e^{3 i pi/8}
    B, A, AB = M.block_tw(0, 0)
    assert np.allclose([B, A, AB], np.exp(1j * np.pi * np.array([1, 2, 3]) / 8))


def _exact(d, k):
    return sum(np.array(M.negacyclic(d[r], k[r]), dtype=object) for r in range(len(d)))


def test_product_exact_random_and_adversarial():
    rng = np.random.default_rng(7)
    N = 2 * M.n
    d = rng.integers(-64, 65, (12, N))
    k = rng.integers(-2**24, 2**24 + 1, (12, N))
    got = M.product(d, k)
    want = _exact(d, k)
    assert np.array_equal(np.rint(got).astype(np.int64).astype(object), want)
    assert np.max(np.abs(got - want.astype(np.float64))) < 0.05
    # adversarial: every term of output coefficient c at its maximum with one sign (|coef| ~ 2^44.6)
    for c in (0, 1023, 2047):
        kk = rng.choice([-2**24, 2**24], (12, N))
        j = np.arange(N)
        src = (c - j) % N
        sign = np.where(j <= c, 1, -1)
        dd = 64 * sign[None, :] * np.sign(kk[:, src])
        got = M.product(dd, kk)
        want = _exact(dd, kk)
        err = np.max(np.abs(got - want.astype(np.float64)))
        assert abs(float(want[c])) > 2**44 and err < 0.1, (c, err)
        assert np.array_equal(np.rint(got).astype(np.int64).astype(object), want)


def test_exchange_regions():
    """br2f_kernel runs each wave-local exchange in the wave's own quarter of the transform's
    cross-wave buffer X (no separate W buffer, round 5). Safe because every exchange direction puts
    wave w's points at slots whose bits 9, 8 equal w on its own side: the forward cross-wave reads
    (P2, xf) and the inverse cross-wave writes (P2, xi) are own-quarter, and both wave-local
    exchanges (wf, wi) are own-quarter on both sides. So after a forward transform's cross-wave reads
    no other wave touches quarter w of X until the next-but-one transform writes X behind the next
    barrier, and an inverse's wave-local exchange precedes its own-quarter cross-wave writes."""
    import fft2_model as M
    own = {"xf": ("read",), "xi": ("write",), "wf": ("write", "read"), "wi": ("write", "read")}
    for name, sides in own.items():
        sw, (pf, pt) = M.SWIZZLES[name], M.EXCHANGES[name]
        for side in sides:
            p = pf if side == "write" else pt
            assert all((sw(M.idx(p, t, e)) >> 8) == (t >> 6) for t in range(M.T) for e in range(M.E)), (name, side)
    # the other side of a cross-wave exchange spans every quarter (it is cross-wave)
    for name, side, p in (("xf", "write", 1), ("xi", "read", 1)):
        sw = M.SWIZZLES[name]
        assert {sw(M.idx(p, t, e)) >> 8 for t in range(64) for e in range(M.E)} == {0, 1, 2, 3}, (name, side)


def test_tangent_forward_matches_premultiplied():
    """The kernel's tangent-form forward passes (Fft1024::fwd_pass_t) compute the same map as the
    premultiplied ones, to rounding, and invert through the unchanged inverse."""
    rng = np.random.default_rng(19)
    z = rng.standard_normal(M.n) + 1j * rng.standard_normal(M.n)
    a, b = M.forward(z, tangent=False), M.forward(z, tangent=True)
    assert np.max(np.abs(a - b)) < 1e-12 * np.max(np.abs(a))
    assert np.max(np.abs(M.inverse(b) / M.n - z)) < 1e-12
