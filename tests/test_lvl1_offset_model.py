"""Integer models of br1f's accumulator representation (tfhe-omr_amd/csrc/br1_fft.hpp, Lvl1Off and
Lvl1Int::round_mod), in numpy with explicit u32 wrap-around, against the plain definitions:

- ac'' = ac + H/2 (mod Q) in [0, Q); the stored negacyclic half n = H - ac'' (signed u32);
- the digits of the word from a rotated entry x'' (either half) and the lane's own n equal
  those of Lvl1Int::digits(canon(x - ac)), i.e. the NonPowOf2ApproxSignedBasis digits (logB 5, d 4, drop 7)
  of the reference's decomposition (detector.rs:553-557 via the level-1 parameters);
- round_mod(y) in [0, Q] with round_mod(y) = round(y) mod Q, and add(ac'', r) = ac'' + r (mod Q)
  in [0, Q), for FFT outputs y = integer + e (|y| < 2^43, |e| < 0.1), including the multiples of q;
- and br2f's level-2 digit words (Digits2S: two's-complement fields, one v_bfe_i32 per digit) give
  the same six digits as Digits2 (detect_kernels.hpp) over the whole canonical range of q2.
"""
import numpy as np

Q = 134215681
H = (Q - 1) // 2
HH = H // 2
M32 = (1 << 32) - 1
DROP, LOGB, D = 7, 5, 4
BIAS = ((1 << (LOGB * (D - 1))) - 1) // ((1 << LOGB) - 1) * (1 << (LOGB - 1))


def u32(x):
    return np.asarray(x, dtype=np.int64) & M32


def s32(x):
    x = u32(x)
    return np.where(x >= 1 << 31, x - (1 << 32), x)


def canon(x):
    x = np.asarray(x, dtype=np.int64) % Q
    return np.where(x > H, x - Q, x)


def ref_digits(v):  # Lvl1Int::digits on a canonical residue
    return u32((((v + (1 << (DROP - 1))) >> DROP) + BIAS) ^ BIAS)


def digit(w, k):  # Lvl1Int::digit: signed field k
    w = u32(w)
    if k < D - 1:
        f = (w >> (LOGB * k)) & 31
        return np.where(f >= 16, f - 32, f)
    return s32(w) >> (LOGB * (D - 1))


def enc(v):
    y = u32(v + HH)
    return np.minimum(y, u32(y + Q))


def dec(a):
    return canon(s32(a) - HH)


def neg(a):
    return u32(H - a)


def off_digits(xs, n):  # Lvl1Off::digits_u: the word shifted left by DROP (low bits: remainder)
    t = u32(xs + n)
    y = np.minimum(np.minimum(t, u32(t + Q)), u32(t - Q))
    C = (1 << (DROP - 1)) - H + (BIAS << DROP)
    return u32(u32(y + C) ^ (BIAS << DROP))


def off_digit(w, k):  # a signed bit-field extract at offset DROP + 5k
    w = u32(w)
    if k < D - 1:
        f = (w >> (DROP + LOGB * k)) & 31
        return np.where(f >= 16, f - 32, f)
    return s32(w) >> (DROP + LOGB * (D - 1))


def off_digit_shifts(w, k):  # Lvl1Off::digit_shifts_u
    w = u32(w)
    s1 = 32 - DROP - LOGB * (k + 1) if k < D - 1 else 0
    s2 = 32 - LOGB if k < D - 1 else DROP + LOGB * (D - 1)
    return s32(u32(w << s1)) >> s2


def round_mod(y):
    k = np.floor(y * (1.0 / Q))
    r = -k * Q + y  # exact for |y| < 2^43 (the fma of the kernel)
    s = r + 6755399441055744.0
    return s.view(np.uint64).astype(np.int64) & M32


def add(a, r):
    s = u32(a + r)
    return np.minimum(s, u32(s - Q))


def test_representation_round_trip():
    v = np.concatenate([np.arange(-H, -H + 1000), np.arange(-500, 500), np.arange(H - 1000, H + 1),
                        np.random.default_rng(1).integers(-H, H + 1, 200000)])
    a = enc(v)
    assert np.all((a >= 0) & (a < Q))
    assert np.array_equal(dec(a), v)
    assert np.array_equal(canon(s32(neg(a)) - HH), canon(-v))  # the stored half is "-ac + H/2"


def test_digit_words_match_the_decomposition():
    rng = np.random.default_rng(2)
    edge = np.array([-H, -H + 1, -1, 0, 1, H - 1, H, HH, -HH, 63, 64, -64, -65])
    x = np.concatenate([rng.integers(-H, H + 1, 400000), np.repeat(edge, len(edge))])
    ac = np.concatenate([rng.integers(-H, H + 1, 400000), np.tile(edge, len(edge))])
    n = neg(enc(ac))
    for xs in (enc(x), neg(enc(-x))):  # x read from the first half, or -x's entry in the second
        got = off_digits(xs, n)
        want = ref_digits(canon(x - ac))
        assert np.array_equal(u32(s32(got) >> DROP), want)  # Lvl1Off::digits (br1f)
        for k in range(D):  # Lvl1Off::digits_u + digit_shifts_u (br1l)
            assert np.array_equal(off_digit_shifts(got, k), digit(want, k))
            assert np.array_equal(off_digit(got, k), digit(want, k))
    # and the digits recompose the rounded value (the basis of detector.rs's decomposition)
    w = ref_digits(canon(x - ac))
    val = sum(digit(w, k) * (32 ** k) for k in range(D))
    assert np.array_equal(val, (canon(x - ac) + 64) >> DROP)
    assert np.all(np.abs(np.stack([digit(w, k) for k in range(D)])) <= 17)


def test_round_mod_and_update():
    rng = np.random.default_rng(3)
    ints = np.concatenate([rng.integers(-(1 << 43), 1 << 43, 300000),
                           np.arange(-40, 41) * Q, np.arange(-40, 41) * Q + 1, np.arange(-40, 41) * Q - 1,
                           np.array([(1 << 43) - 1, -(1 << 43) + 1])])
    for e in (0.0, 0.0999, -0.0999, 0.03):
        y = ints.astype(np.float64) + e
        r = round_mod(y)
        assert np.all((r >= 0) & (r <= Q))
        assert np.array_equal(r % Q, ints % Q)
    a = enc(rng.integers(-H, H + 1, ints.size))
    r = round_mod(ints.astype(np.float64) - 0.05)
    got = add(a, r)
    assert np.all((got >= 0) & (got < Q))
    assert np.array_equal(dec(got), canon(dec(a) + ints))


# ---- level 2: br2f's signed-field digit words (Digits2S, tfhe-omr_amd/csrc/br2_fft.hpp) --------
def _digits2_ref(v):
    """Digits2 (detect_kernels.hpp): biased 7-bit fields (the top one 8 bits wide), minus 64."""
    y = np.floor(v / 256.0 + 0.5) + 2216338399296.0  # v / 256 is exact: the kernel's fma
    hi = np.floor(y * (1.0 / 2097152.0))
    lo = y - hi * 2097152.0
    w = [lo.astype(np.int64), hi.astype(np.int64)]
    out = []
    for k in range(6):
        h, j = divmod(k, 3)
        width = 8 if j == 2 else 7
        out.append(((w[h] >> (7 * j)) & ((1 << width) - 1)) - 64)
    return np.stack(out)


def _digits2s(v):
    """Digits2S::pack: the words are the low dword and bits 21..52 of the FP64 pattern of
    y + 64 (1 + 128 + .. + 128^4) + 1.5 * 2^52 (exact)."""
    y = np.floor(v / 256.0 + 0.5) + (17315143744.0 + 6755399441055744.0)
    b = y.view(np.uint64)
    w0 = u32((b & np.uint64(0xFFFFFFFF)).astype(np.int64)) ^ 0x102040
    w1 = u32(((b >> np.uint64(21)) & np.uint64(0xFFFFFFFF)).astype(np.int64)) ^ 0x2040
    out = []
    for k in range(6):
        h, j = divmod(k, 3)
        w = s32(w0 if h == 0 else w1)
        width = 16 if (h == 1 and j == 2) else 7
        f = (w >> (7 * j)) & ((1 << width) - 1)
        out.append(np.where(f >= 1 << (width - 1), f - (1 << width), f))
    return np.stack(out)


def test_level2_signed_digit_fields_match_digits2():
    Q2 = 1125899906826241  # SecondLevelField, see tfhe-omr_amd/csrc/common.hpp OMR_Q2
    h2 = Q2 // 2
    rng = np.random.default_rng(4)
    v = np.concatenate([rng.integers(-h2, h2 + 1, 300000), np.array([-h2, h2, 0, 1, -1, 127, 128, -128, -129]),
                        np.arange(-2000, 2000) * 256 + 128]).astype(np.float64)
    assert np.array_equal(_digits2s(v), _digits2_ref(v))
    d = _digits2s(v)
    assert np.array_equal(sum(d[k] * 128 ** k for k in range(6)), np.floor(v / 256.0 + 0.5).astype(np.int64))


def test_level2_limb_update_exact():
    """limb_acc (br2_fft.hpp): acc + lo + 2^25 hr -> the exact centred residue mod q2, in FP64 as the
    kernel computes it (one quotient, one fma, one red), against Python integers."""
    Q2 = 1125899906826241
    q = float(Q2)
    qinv = 1.0 / q
    limb = 33554432.0
    rng = np.random.default_rng(11)
    n = 200000
    h2 = Q2 // 2
    acc = rng.integers(-h2, h2 + 1, n).astype(np.float64)
    lim = 2 ** 46 - 1
    lo = rng.integers(-lim, lim + 1, n).astype(np.float64)
    hr = rng.integers(-lim, lim + 1, n).astype(np.float64)
    edge = np.array([-h2, h2, 0, 1, -1], dtype=np.float64)
    acc = np.concatenate([acc, np.repeat(edge, 9)])
    lo = np.concatenate([lo, np.tile(np.array([-lim, lim, 0], dtype=np.float64), 15)])
    hr = np.concatenate([hr, np.tile(np.array([lim, -lim, 0], dtype=np.float64).repeat(3), 5)])

    def red(x):
        return _fma(-np.rint(x * qinv), q, x)

    x = acc + lo
    hi = hr * limb
    k = np.rint(_fma(hr, limb * qinv, x * qinv))
    got = red(_fma(-k, q, hi) + x)
    for a, l, h, g in zip(acc.astype(np.int64), lo.astype(np.int64), hr.astype(np.int64), got):
        want = (int(a) + int(l) + (int(h) << 25)) % Q2
        if want > h2:
            want -= Q2
        assert int(g) == want and float(int(g)) == g


def _fma(a, b, c):
    """Correctly rounded a * b + c elementwise (exact rational arithmetic, then one rounding)."""
    from fractions import Fraction
    a, b, c = np.broadcast_arrays(np.asarray(a, np.float64), np.asarray(b, np.float64), np.asarray(c, np.float64))
    return np.array([float(Fraction(x) * Fraction(y) + Fraction(z)) for x, y, z in zip(a.ravel(), b.ravel(), c.ravel())]).reshape(a.shape)


def _trace_digits_recursive(v):
    """DigitsTrace's reference: d = y - 4 floor(y / 4 + 1/2), 24 times, then the rest (the oracle's
    recursive NonPowOf2ApproxSignedBasis form for base 4, 25 digits)."""
    y = v.copy()
    out = []
    for _ in range(24):
        c = np.floor(y * 0.25 + 0.5)
        out.append((y - 4 * c).astype(np.int64))
        y = c
    out.append(y.astype(np.int64))
    return np.stack(out)


def _trace_digits_closed(v):
    """DigitsTrace::pack / get_int (detect_kernels.hpp): the dwords of v + 2 (1 + .. + 4^23) + 1.5 2^52
    with every 2-bit field XORed with 2, two's-complement 2-bit fields, the top one 3 bits at 48."""
    b = (v + (187649984473770.0 + 6755399441055744.0)).view(np.uint64)
    w0 = s32(u32((b & np.uint64(0xFFFFFFFF)).astype(np.int64)) ^ 0xAAAAAAAA)
    w1 = s32(u32((b >> np.uint64(32)).astype(np.int64)) ^ 0xAAAA)
    out = []
    for k in range(25):
        w, off, width = (w0, 2 * k, 2) if k < 16 else (w1, 2 * (k - 16), 3 if k == 24 else 2)
        f = (w >> off) & ((1 << width) - 1)
        out.append(np.where(f >= 1 << (width - 1), f - (1 << width), f))
    return np.stack(out)


def test_trace_digit_closed_form_matches_recursive():
    Q2 = 1125899906826241
    h2 = Q2 // 2
    rng = np.random.default_rng(5)
    v = np.concatenate([rng.integers(-h2, h2 + 1, 300000), np.array([-h2, h2, 0, 1, -1, 2, -2, 3, -3]),
                        np.arange(-3000, 3000) * 4 ** 12 + 2 * (4 ** 12 - 1) // 3]).astype(np.float64)
    d = _trace_digits_closed(v)
    assert np.array_equal(d, _trace_digits_recursive(v))
    assert np.array_equal(sum(d[k] * 4 ** k for k in range(25)), v.astype(np.int64))
