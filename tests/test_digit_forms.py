"""The closed-form gadget digits used by the kernels (br1_fft.hpp Lvl1Int::digits/digit,
detect_kernels.hpp Digits2) equal the recursive signed decomposition of the oracle
(NonPowOf2ApproxSignedBasis: y = floor((v + 2^(drop-1)) / 2^drop), balanced digits, unbounded
top digit) on boundary and random canonical residues."""
import numpy as np

import oracle_lib as O

Q1, Q2 = 134215681, 1125899906826241


def _recursive(v, logb, d, drop):
    y = (v + (1 << (drop - 1))) >> drop
    out = []
    for _ in range(d - 1):
        c = (y + (1 << (logb - 1))) >> logb
        out.append(y - (c << logb))
        y = c
    out.append(y)
    return out


def _residues(q, n, seed):
    h = (q - 1) // 2
    rng = np.random.default_rng(seed)
    return np.concatenate([rng.integers(-h, h + 1, n), np.arange(-h, -h + 3000), np.arange(h - 3000, h + 1),
                           np.arange(-70000, 70000)]).astype(np.int64)


def test_level1_closed_form_digits():
    v = _residues(Q1, 500_000, 1)
    bias = ((1 << 15) - 1) // 31 * 16  # 16 (1 + 32 + 32^2)
    yb = (((v + 64) >> 7) + bias).astype(np.int64) & 0xFFFFFFFF  # uint32 word as on the device
    signed = np.where(yb >= 1 << 31, yb - (1 << 32), yb)
    closed = [((yb >> (5 * k)) & 31) - 16 for k in range(3)] + [signed >> 15]
    for a, b in zip(_recursive(v, 5, 4, 7), closed):
        assert np.array_equal(a, b)
    # the word the kernel keeps (Lvl1Int::digits): yb ^ bias, each digit one signed bit-field
    # of width 5 at offset 5k (k < 3) or 17 at offset 15 (top digit); the kernel extracts it with
    # two uniform shifts, (int)(w << (32 - off - width)) >> (32 - width)
    w = yb ^ bias
    ws = np.where(w >= 1 << 31, w - (1 << 32), w)

    def sbfe(x, off, width):
        f = (x >> off) & ((1 << width) - 1)
        return np.where(f >= 1 << (width - 1), f - (1 << width), f)

    extracted = [sbfe(w, 5 * k, 5) for k in range(3)] + [sbfe(ws & 0xFFFFFFFF, 15, 17)]
    for a, b in zip(_recursive(v, 5, 4, 7), extracted):
        assert np.array_equal(a, b)


def test_level2_closed_form_digits():
    v = _residues(Q2, 500_000, 2)
    # detect_kernels.hpp Digits2: bias 64 (1 + 128 + ... + 128^5), exact in FP64 (0 <= y' < 2^43)
    y = np.floor(v.astype(np.float64) / 256 + 0.5) + 2216338399296.0
    assert y.min() >= 0 and y.max() < 2.0 ** 43
    hi = np.floor(y / 2097152.0)
    lo = (y - hi * 2097152.0).astype(np.int64)
    hi = hi.astype(np.int64)
    assert lo.max() < 1 << 21 and hi.max() < 1 << 22
    # field j of either word: offset 7 j, width 7 (j < 2) or 8 (j = 2; bit 21 of lo is zero)
    field = lambda w, j: (w >> (7 * j)) & (255 if j == 2 else 127)
    closed = [field(lo, j) - 64 for j in range(3)] + [field(hi, j) - 64 for j in range(3)]
    for a, b in zip(_recursive(v, 7, 6, 8), closed):
        assert np.array_equal(a, b)


def test_recursive_form_is_the_oracle_decomposition():
    rng = np.random.default_rng(3)
    for which, q, basis in ((1, Q1, (5, 4, 7)), (2, Q2, (7, 6, 8))):
        for u in rng.integers(0, q, 300).tolist() + [0, 1, q - 1, (q - 1) // 2, (q + 1) // 2]:
            c = u - q if u > (q - 1) // 2 else u
            digits = np.zeros(8, np.int64)
            n = O.lib().oref_decompose(which, int(u), digits)
            assert n == basis[1]
            assert [int(x[0]) for x in _recursive(np.array([c]), *basis)] == digits[:n].tolist()
