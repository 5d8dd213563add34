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
    assert e1 < 0.15 and e2 < 0.45, (e1, e2)
    assert 5e6 < k1 < 2e7 and 1e6 < k2 < 3e6  # ~4 sigma of uniform keys' spectra
