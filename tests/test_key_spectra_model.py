"""The double-double key transform (tfhe-omr_amd/csrc/key_spectra.hpp) is a radix-2 Cooley-Tukey
tree in natural index order; the FFT kernels run the same tree in radix-8/4/2 passes with
permuted register/lane layouts. This checks, in complex128 on CPU, that the tree restated here
(as key_spectrum_dd_kernel runs it) returns at every index exactly the value the kernels' pass
models return there: level 1 against tools/fft_exactness.py's Fft8P (WgFft<64, 8, 9>), level 2
against tests/fft2_model.py (Fft1024, P4 layout). With that, the stored key spectra line up with
the digit spectra, and the a priori bound's |K^ - K| <= u |K| applies to the values the
multiply-accumulate reads."""
import os
import sys

import numpy as np

import fft2_model as M2

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import fft_exactness as FX  # noqa: E402


def tree_fft(z, L):
    """key_spectrum_dd_kernel's loop: stage s splits on index bit L-1-s, node i = top s bits,
    W(s, i) = w^(eps(s, i) / 2), w = exp(i pi / 2n), butterfly (x_j + W x_j', x_j - W x_j')."""
    n = 1 << L
    x = np.array(z, dtype=np.complex128).reshape(1, n)
    eps = [n]
    for s in range(L):
        h = 1 << (L - 1 - s)
        half = np.array([e // 2 for e in eps])
        w = np.exp(1j * np.pi * (half % (4 * n)) / (2 * n))
        xv = x.reshape(1, 1 << s, 2, h)
        v = w[None, :, None] * xv[:, :, 1, :]
        a, b = xv[:, :, 0, :] + v, xv[:, :, 0, :] - v
        xv[:, :, 0, :], xv[:, :, 1, :] = a, b
        eps = [y for e in eps for y in ((e // 2) % (4 * n), (e // 2 + 2 * n) % (4 * n))]
    return x[0]


def test_tree_matches_level1_passes():
    rng = np.random.default_rng(11)
    f = FX.Fft8P()
    for _ in range(3):
        z = rng.integers(-2 ** 26, 2 ** 26, 512) + 1j * rng.integers(-2 ** 26, 2 ** 26, 512)
        want = f.fwd(z)
        got = tree_fft(z, 9)
        assert np.max(np.abs(got - want)) <= 1e-12 * np.max(np.abs(want))


def test_tree_matches_level2_passes():
    rng = np.random.default_rng(12)
    for _ in range(2):
        z = rng.integers(-2 ** 24, 2 ** 24, 1024) + 1j * rng.integers(-2 ** 24, 2 ** 24, 1024)
        want = M2.forward(z)          # [256][4], register e of thread t holds index IDX[4][t][e]
        got = tree_fft(z, 10)[M2.IDX[4]]
        assert np.max(np.abs(got - want)) <= 1e-12 * np.max(np.abs(want))


def test_tree_inverse_gives_negacyclic_product():
    """Products of tree spectra invert (conjugate tree, unscaled) to the exact negacyclic product:
    the evaluation points of the tree are the roots of X^n - i in the folded ring."""
    rng = np.random.default_rng(13)
    n, L = 1024, 10
    a = rng.integers(-64, 65, 2 * n)
    k = rng.integers(-2 ** 24, 2 ** 24, 2 * n)
    A_, K_ = tree_fft(M2.fold(a.astype(float)), L), tree_fft(M2.fold(k.astype(float)), L)
    # inverse through the fft2 model (P4 layout in, natural order out, x1024)
    prod = M2.inverse((A_ * K_ / n)[M2.IDX[4]])
    got = np.rint(M2.unfold(prod)).astype(np.int64)
    want = np.array(M2.negacyclic(a, k), dtype=np.int64)
    assert np.array_equal(got, want)


def test_apriori_bound_proves_both_levels_exact_on_the_bench_key():
    """On bench.py's key (pack 42, key seed 7) the a priori bound is below 0.5 for both levels, so
    rounding every FFT product coefficient recovers the exact integer for every input
    (the library evaluates the same bound on its stored spectra, checked against
    this restatement in tests/test_gpu_exactness.py)."""
    import product_lib as PL
    from fft_bound import apriori_bounds
    e1, e2, k1, k2 = apriori_bounds(PL.keys()[2])
    assert e1 < 0.15 and e2 < 0.47, (e1, e2)  # 0.136, 0.445 (round 5: tangent-form forward passes)
    assert 5e6 < k1 < 2e7 and 1e6 < k2 < 3e6  # ~4 sigma of uniform keys' spectra
    from fft_bound import apriori_bound_latency2
    ey = apriori_bound_latency2(PL.keys()[2])
    assert ey < e2, (ey, e2)  # the latency path's shorter chains (br2y_kernel) round less


def test_double_double_twiddles_match_long_double():
    """The library's double-double twiddles (host code of the key transform, no GPU) equal
    exp(i pi h / 2n) of the tree (eps recursion) to within long double's own accuracy, and each
    double-double is normalised (|lo| <= ulp(hi) / 2)."""
    import product_lib as PL
    A = PL.omr_amd
    pi = np.arctan(np.longdouble(1)) * 4
    for level, L in ((1, 9), (2, 10)):
        n = 1 << L
        tw = A.fft_twiddles_dd(level)
        half, eps = [], [n]
        for s in range(L):
            half += [e // 2 for e in eps]
            eps = [y for e in eps for y in ((e // 2) % (4 * n), (e // 2 + 2 * n) % (4 * n))]
        ang = pi * np.array(np.array(half) % (4 * n), dtype=np.longdouble) / np.longdouble(2 * n)
        re = tw[:, 0].astype(np.longdouble) + tw[:, 1].astype(np.longdouble)
        im = tw[:, 2].astype(np.longdouble) + tw[:, 3].astype(np.longdouble)
        assert np.max(np.abs(re - np.cos(ang))) < 2e-18 and np.max(np.abs(im - np.sin(ang))) < 2e-18
        for c in (0, 2):
            assert np.all(np.abs(tw[:, c + 1]) <= np.spacing(np.abs(tw[:, c])) / 2 + 1e-300)


def _dd_two_sum(a, b):
    s = a + b
    bb = s - a
    return s, (a - (s - bb)) + (b - bb)


def _dd_quick(a, b):
    s = a + b
    return s, b - (s - a)


def _dd_add(ah, al, bh, bl):
    sh, sl = _dd_two_sum(ah, bh)
    th, tl = _dd_two_sum(al, bl)
    sl = sl + th
    sh, sl = _dd_quick(sh, sl)
    sl = sl + tl
    return _dd_quick(sh, sl)


def _two_prod(a, b):
    p = a * b
    # Dekker split (no fma in numpy): exact error of the product
    c = 134217729.0
    def split(x):
        t = c * x
        hi = t - (t - x)
        return hi, x - hi
    ah, al = split(a)
    bh, bl = split(b)
    return p, ((ah * bh - p) + ah * bl + al * bh) + al * bl


def _dd_mul(ah, al, bh, bl):
    p, e = _two_prod(ah, bh)
    e = e + (ah * bl + al * bh)
    return _dd_quick(p, e)


def test_double_double_tree_meets_the_storage_bound():
    """key_spectrum_dd_kernel's arithmetic (exactness.hpp dd_add / dd_mul, the tree of dd_tree_fft)
    replayed in numpy float64 on key-sized rows with the library's twiddles: rounded once, every
    spectral value is within u |K| (1 + 2^-10) of a long-double evaluation -- the storage term
    u' = u (1 + 2^-40) of the a priori bound up to the reference's own accuracy."""
    import product_lib as PL
    A = PL.omr_amd
    rng = np.random.default_rng(5)
    pi = np.arctan(np.longdouble(1)) * 4
    for level, L, lim in ((1, 9, 2 ** 26), (2, 10, 2 ** 24)):
        n = 1 << L
        tw = A.fft_twiddles_dd(level)
        z = rng.integers(-lim, lim, (4, 2 * n)).astype(np.float64)
        rh, ih = z[:, :n].copy(), z[:, n:].copy()
        rl, il = np.zeros_like(rh), np.zeros_like(ih)
        for s in range(L):
            h = 1 << (L - 1 - s)
            blk = np.arange(n // 2) >> (L - 1 - s)
            j = (blk << (L - s)) | (np.arange(n // 2) & (h - 1))
            j1 = j + h
            w = tw[(1 << s) - 1 + blk]
            # v = w * x1 (complex double-double)
            a1 = _dd_mul(w[:, 0], w[:, 1], rh[:, j1], rl[:, j1])
            a2 = _dd_mul(w[:, 2], w[:, 3], ih[:, j1], il[:, j1])
            vr = _dd_add(a1[0], a1[1], -a2[0], -a2[1])
            b1 = _dd_mul(w[:, 0], w[:, 1], ih[:, j1], il[:, j1])
            b2 = _dd_mul(w[:, 2], w[:, 3], rh[:, j1], rl[:, j1])
            vi = _dd_add(b1[0], b1[1], b2[0], b2[1])
            x0 = (rh[:, j].copy(), rl[:, j].copy(), ih[:, j].copy(), il[:, j].copy())
            rh[:, j], rl[:, j] = _dd_add(x0[0], x0[1], vr[0], vr[1])
            ih[:, j], il[:, j] = _dd_add(x0[2], x0[3], vi[0], vi[1])
            rh[:, j1], rl[:, j1] = _dd_add(x0[0], x0[1], -vr[0], -vr[1])
            ih[:, j1], il[:, j1] = _dd_add(x0[2], x0[3], -vi[0], -vi[1])
        # long-double reference of the same tree (twiddles from the eps recursion)
        x = (z[:, :n] + 1j * z[:, n:]).astype(np.clongdouble)
        eps = [n]
        for s in range(L):
            h = 1 << (L - 1 - s)
            half = np.array([e // 2 for e in eps])
            ang = pi * np.array(half % (4 * n), dtype=np.longdouble) / np.longdouble(2 * n)
            wv = np.cos(ang) + 1j * np.sin(ang)
            xv = x.reshape(4, 1 << s, 2, h)
            v = wv[None, :, None] * xv[:, :, 1, :]
            a, b = xv[:, :, 0, :] + v, xv[:, :, 0, :] - v
            xv[:, :, 0, :], xv[:, :, 1, :] = a, b
            eps = [y for e in eps for y in ((e // 2) % (4 * n), (e // 2 + 2 * n) % (4 * n))]
        K = x / n
        got = (rh + 1j * ih).astype(np.clongdouble) / n
        err = np.abs(got - K)
        assert np.all(err <= 2.0 ** -53 * np.abs(K) * (1 + 2 ** -10) + 1e-17 * np.abs(K).max()), (level, err.max())
