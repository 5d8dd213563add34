"""Crafted evaluation keys for the exactness contract (test infrastructure).

The a priori bound E (tests/fft_bound.py) grows with kappa, the largest magnitude
of a key row's spectrum. Uniform key rows peak near 4 sigma; a row whose coefficients all lean
into one spectral point reaches the largest magnitude a centred 25-bit limb allows. This rewrites
the level-2 rows (BSK2, [670][12][2][2048] canonical u64) of a few steps so that the low limb of
every row and output is +-(2^24 - 1) with the signs aligned to spectral point 0 of the folded,
twisted transform z_k = p_k + i p_{k+1024}, K[0] = (1/n) sum_k z_k e^{i pi k / 2n}: then
Re(z_k e^{i pi k / 2n}) = (2^24 - 1)(|cos| + |sin|) for every k and K[0] ~ 1.27 (2^24 - 1), about
11x the uniform rows' kappa, which puts E2 well above 1. The key stays a valid operand of the
detect path (any canonical residues are), so the GPU output is checked against the oracle on it.
"""
import numpy as np

Q1 = 134215681
Q2 = 1125899906826241
LIMB_MAX = (1 << 24) - 1
H1 = (Q1 - 1) // 2


def aligned_row(n=1024, peak=LIMB_MAX):
    """A coefficient-domain row (2n centred values of magnitude `peak`) whose folded spectrum peaks
    at point 0."""
    phi = np.pi * np.arange(n) / (2 * n)
    re = np.where(np.cos(phi) >= 0, peak, -peak)
    im = np.where(np.sin(phi) >= 0, -peak, peak)  # Re(i v e^{i phi}) = -v sin(phi)
    return np.concatenate([re, im]).astype(np.int64)


def high_kappa_bsk1(bsk1, steps=(0, 1, 2, 3)):
    """Level 1 the same way (round 5): a copy of bsk1 (u32 [512][8][2][1024]) with every row and
    output of `steps` set to the aligned row of peak (q1 - 1) / 2, the largest centred residue: the
    folded 512-point spectrum then peaks at 4 / pi * 512 * (q1 - 1) / 2, about 24x a uniform row's,
    which puts E1 above 1."""
    out = np.array(bsk1, dtype=np.uint32, copy=True).reshape(512, 8, 2, 1024)
    row = aligned_row(512, H1)
    canon = np.where(row < 0, row + Q1, row).astype(np.uint32)
    for i in steps:
        out[i, :, :, :] = canon[None, None, :]
    return out.reshape(np.shape(bsk1))


def high_kappa_bsk2(bsk2, steps=(0, 1, 2, 3)):
    """A copy of bsk2 (u64 [670][12][2][2048]) with every row and output of `steps` aligned."""
    out = np.array(bsk2, dtype=np.uint64, copy=True).reshape(670, 12, 2, 2048)
    row = aligned_row()
    canon = np.where(row < 0, row + Q2, row).astype(np.uint64)
    for i in steps:
        out[i, :, :, :] = canon[None, None, :]
    return out.reshape(np.shape(bsk2))
