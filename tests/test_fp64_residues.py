"""The FP64 residue canonicalisation the kernels use (device_ntt.hpp canon / canon_small with
OMR_CANON_RED, br1_fft.hpp Lvl1Int::canon with BR1F_CANON_MIN), replayed in numpy with the
device's IEEE operations: red(x) = x - rint(x * fl(1/q)) * q (the product q * rint(...) and the
difference are exact in FP64 here, as the device's fma is), rint = round half to even.

Claims checked at both primes:
  * red(x) is the exact centred representative for every integer |x| <= q - 1 (sums and
    differences of two canonical residues), including the +-(q-1)/2, +-(q+1)/2 boundaries;
  * red(red(x)) is the exact centred representative for integers |x| < 2^53.
and the int32 unsigned-min fold of the level-1 accumulator update."""
import numpy as np

Q1, Q2 = 134215681, 1125899906826241


def _red(x, q):
    x = np.asarray(x, dtype=np.float64)
    qinv = np.float64(1.0) / np.float64(q)
    return x - np.rint(x * qinv) * np.float64(q)


def _centred(x, q):
    r = np.mod(x, q)
    return np.where(r > (q - 1) // 2, r - q, r)


def test_red_canonicalises_sums_of_canonical_residues():
    rng = np.random.default_rng(11)
    for q in (Q1, Q2):
        h = (q - 1) // 2
        xs = np.concatenate([np.arange(h - 20000, h + 20001), np.arange(-h - 20000, -h + 20001),
                             np.arange(q - 20000, q), np.arange(-q + 1, -q + 20001),
                             rng.integers(-(q - 1), q, 400_000)]).astype(np.int64)
        xs = xs[np.abs(xs) <= q - 1]
        got = _red(xs.astype(np.float64), q)
        assert np.array_equal(got.astype(np.int64), _centred(xs, q))
        assert np.all(np.abs(got) <= h)


def test_double_red_canonicalises_below_2_53():
    rng = np.random.default_rng(12)
    for q in (Q1, Q2):
        xs = rng.integers(-(1 << 53) + 1, 1 << 53, 400_000, dtype=np.int64)
        # values next to multiples of q plus/minus half: where a single rint can land one off
        k = rng.integers(-(1 << 53) // q + 1, (1 << 53) // q - 1, 50_000, dtype=np.int64)
        edge = np.concatenate([k * q + (q - 1) // 2 + d for d in (-2, -1, 0, 1, 2, 3)])
        xs = np.concatenate([xs, edge])
        got = _red(_red(xs.astype(np.float64), q), q)
        assert np.array_equal(got.astype(np.int64), _centred(xs, q))


def test_level1_unsigned_min_canon():
    q, h = Q1, (Q1 - 1) // 2
    rng = np.random.default_rng(13)
    x = np.concatenate([rng.integers(-q - h + 1, q + h, 400_000), np.arange(-q - h + 1, -q - h + 2000),
                        np.arange(q + h - 2000, q + h), np.arange(-h - 2000, -h + 2000),
                        np.arange(h - 2000, h + 2000)]).astype(np.int64)
    y = (x + h) & 0xFFFFFFFF
    y = np.minimum(y, (y + q) & 0xFFFFFFFF)
    y = np.minimum(y, (y - q) & 0xFFFFFFFF)
    got = y.astype(np.int64) - h
    assert np.array_equal(got, _centred(x, q))


def _mm_bound(a):
    """|mm(a, w)| / q for |a| <= A q, |w| <= (q - 1) / 2 (device_ntt.hpp mm): the quotient
    rint(fl(h * fl(1/q))) errs by at most 0.5 + 2^-52 |h / q| (three roundings), and the low part l
    of the error-free product adds |h| 2^-53: with q < 2^50 that is (0.5 + 0.125 A + 0.0625 A)."""
    return 0.5 + 0.1875 * a


def _replay_mm(bound, seed):
    """mm on operands up to bound * q: exact residue, no intermediate above 2^53, within _mm_bound."""
    q = Q2
    rng = np.random.default_rng(seed)
    n = 20_000
    a = np.rint(rng.uniform(-bound, bound, n) * q)
    a[:2] = (-np.floor(bound * q), np.floor(bound * q))
    w = rng.integers(-(q - 1) // 2, (q - 1) // 2 + 1, n).astype(np.float64)
    w[:2] = ((q - 1) // 2, (q - 1) // 2)
    h = a * w                        # rounded product
    qe = np.rint(h * (1.0 / q))      # rint(h * fl(1/q))
    # l = fma(a, w, -h) and fma(-qe, q, h) are exact on the device; replay with Python ints
    for x, y, hh, e in zip(a.astype(np.int64), w.astype(np.int64), h, qe):
        x, y, hh, e = int(x), int(y), int(hh), int(e)
        r = (hh - e * q) + (x * y - hh)
        assert abs(hh - e * q) < 2**53 and abs(r) < 2**53
        assert r % q == (x * y) % q
        assert abs(r) <= _mm_bound(bound) * q


def _stage(a_u, a_v):
    """CT butterfly u +- mm(v, w): the output bound from the operand bounds."""
    return a_u + _mm_bound(a_v)


def test_level2_forward_ntt_bound_with_stage01_tables():
    """device_ntt.hpp CmuxNtt::fwd_small: after stages 0 and 1 from the tables (each entry
    canonical) |x| <= |d| + 3 (q - 1) / 2 <= 1.5q + 64; stages 2..5 each add mm(x, w); before
    stage 6 only the u operands are reduced (|u| <= q/2 + 2), the v operands go into mm as they
    are; stages 6..10 follow. Every value stays below 2^53 = 8q (q2 < 2^50); the mm bound is
    replayed in FP64 at the largest operands (5.62q before stage 6, 6.72q at the output)."""
    q = Q2
    b = 1.5 + 64 / q
    for _ in range(4):  # stages 2, 3, 4, 5
        b = _stage(b, b)
    assert 5.6 < b < 5.63
    red = 0.5 + 2 / q
    b = _stage(red, b)  # stage 6: reduced u, unreduced v
    for _ in range(4):  # stages 7..10
        b = _stage(b, b)
    assert 6.7 < b < 6.73 and b * q < 2.0**53
    _replay_mm(5.63, 14)
    _replay_mm(6.73, 15)
    # the key conversion (CmuxNtt::fwd from canonical residues) has the same shape
    k = 0.5
    for _ in range(6):
        k = _stage(k, k)
    k = _stage(red, k)
    for _ in range(4):
        k = _stage(k, k)
    assert k < 7.0


def test_level2_mac_four_products_per_reduction():
    """detect_kernels.hpp cmux_step3: the forward transform output is |x| <= 6.72q, so each
    product |mm(x, key)| <= 1.76q (|key| <= q/2), and a reduced sum (|acc| <= q/2 + 2) plus four
    products stays below 7.6q < 8q < 2^53. A fifth product would not fit."""
    b = 6.73
    prod = _mm_bound(b)
    assert prod < 1.77
    assert (0.5 + 4 * prod) < 7.6 and (0.5 + 4 * prod) * Q2 < 2.0**53
    assert (0.5 + 5 * prod) * Q2 > 2.0**53


def test_inverse_twiddles_mirror_forward_table():
    """device_ntt.hpp inv_passC<MIRROR>: psi^-brv(2^s + j) = -psi^brv(2^(s+1) - 1 - j) (mod q2) for
    every node of the 2048-point negacyclic table (psi = 22^((q2-1)/4096), 11-bit reversal), so
    the level-2 inverse reads the forward table and multiplies (v - u) instead of (u - v)."""
    q, L = Q2, 11
    psi = pow(22, (q - 1) // 4096, q)
    assert pow(psi, 2048, q) == q - 1

    def brv(k):
        return int(format(k, f"0{L}b")[::-1], 2)

    tw = [pow(psi, brv(k), q) for k in range(1 << L)]
    for s in range(L):
        for j in range(1 << s):
            itw = pow(psi, (4096 - brv((1 << s) + j)) % 4096, q)
            assert itw == (q - tw[(2 << s) - 1 - j]) % q


def test_level1_magic_round_reduce():
    """br1_fft.hpp Lvl1Int::round_red: for y = integer + e (|y| < 2^43, |e| < 0.01, an FFT product
    output), r = y - rint(y / q) q keeps the fraction exactly, and the low 32 bits of r + 1.5 * 2^52
    are round(r) = round(y) mod q (centred, |.| <= (q + 1) / 2) in two's complement."""
    q = Q1
    rng = np.random.default_rng(15)
    n = 400_000
    ints = np.concatenate([rng.integers(-(1 << 43) + 1, 1 << 43, n), np.arange(-3000, 3000),
                           rng.integers(-(1 << 43) // q, (1 << 43) // q, 20_000) * q + (q - 1) // 2])
    e = rng.uniform(-0.01, 0.01, ints.size)
    y = ints.astype(np.float64) + e
    k = np.rint(y * (1.0 / q))
    r = y - k * q  # exact here, as the device's fma
    t = r + 6755399441055744.0
    low = (t.view(np.uint64) & 0xFFFFFFFF).astype(np.int64)
    got = np.where(low >= 1 << 31, low - (1 << 32), low)
    want = _centred(ints, q)
    assert np.all(np.abs(got) <= (q + 1) // 2)
    assert np.array_equal(np.mod(got, q), np.mod(want, q))
