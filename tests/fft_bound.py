"""A priori bound on the rounding error of the FFT external products, restated
from the coefficient-domain key with numpy -- the same formula context.hip's apriori_bound
evaluates on the device-stored double-double key spectra at context creation:

  E = n D (1 + 2^-30) max over steps i and output spectra o of
      [(delta_fwd + delta_inv + u (1 + 2^-40)) sum_r kappa_{i,r,o} + sqrt(2) u sum_k (2R - 2k) kappa_{i,r(k),o}]

n complex points, R GGSW rows accumulated in the order r(0), r(1), ..., D = sqrt(2n) d_max,
delta_fwd + delta_inv = 37u + 32u (level 1) or 41u + 26u (level 2; the forward passes in
tangent form), kappa_{i,r,o} = max_j |K_{i,r,o}[j]| (spectrum of key row r of step i, output o;
level 2: per 25-bit limb). Spectral magnitudes do not depend on the output order, so a plain
twisted DFT gives them: K[m] = (1/n) sum_k z_k e^{i pi k / 2n} e^{2 pi i k m / n}."""
import numpy as np

U = 2.0 ** -53
ORDER2 = [0, 3, 1, 4, 2, 5, 6, 9, 7, 10, 8, 11]  # br2f_kernel's digit issue order


def _centred(v, q):
    v = v.astype(np.int64)
    return np.where(v > (q - 1) // 2, v - q, v).astype(np.float64)


def _row_max(rows, n):
    tw = np.exp(1j * np.pi * np.arange(n) / (2 * n))
    z = rows[..., :n] + 1j * rows[..., n:]
    return np.abs(np.fft.fft(z * tw, axis=-1)).max(axis=-1) / n


def _bound(kmax, n, R, dmax, order, dft, weights=None):
    """kmax [steps][R][outputs]; dft = (delta_fwd + delta_inv) / u; weights: the MAC's rounding
    weight per position of `order` (default: one chain of 2R fmas, 2R - 2k)"""
    k = kmax[:, order, :]
    w = (2.0 * R - 2.0 * np.arange(R) if weights is None else np.asarray(weights, np.float64))[None, :, None]
    inner = (dft * U + U * (1 + 2.0 ** -40)) * k.sum(axis=1) + np.sqrt(2.0) * U * (w * k).sum(axis=1)
    return n * np.sqrt(2.0 * n) * dmax * inner.max() * (1 + 2.0 ** -30)


def apriori_bounds(dk, q1=134215681, q2=1125899906826241):
    """(E1, E2, kappa1, kappa2) for a DetectionKey (omr_amd.DetectionKey layout)."""
    r1 = _centred(dk.bsk1.reshape(512, 8, 2, 1024), q1)
    k1 = _row_max(r1, 512)                                   # [512][8][2]
    r2 = _centred(dk.bsk2.reshape(670, 12, 2, 2048), q2)
    hi = np.rint(r2 / 2.0 ** 25)
    k2 = np.stack([_row_max(r2 - hi * 2.0 ** 25, 1024), _row_max(hi, 1024)], axis=-1).reshape(670, 12, 4)
    e1 = _bound(k1, 512, 8, 16.0, list(range(8)), 37 + 32)
    e2 = _bound(k2, 1024, 12, 64.0, ORDER2, 41 + 26)
    return e1, e2, float(k1.max()), float(k2.max())


def apriori_bound_latency2(dk, q2=1125899906826241):
    """Level 2 as br2y_kernel (the latency path) accumulates it (context.hip, apriori_bound level 3):
    each group chains its three rows (weights 6, 4, 2), then two additions: 8 - 2 j for digit
    3 g + j of either polynomial."""
    r2 = _centred(dk.bsk2.reshape(670, 12, 2, 2048), q2)
    hi = np.rint(r2 / 2.0 ** 25)
    k2 = np.stack([_row_max(r2 - hi * 2.0 ** 25, 1024), _row_max(hi, 1024)], axis=-1).reshape(670, 12, 4)
    return _bound(k2, 1024, 12, 64.0, list(range(12)), 41 + 26, [8 - 2 * ((r % 6) % 3) for r in range(12)])


def apriori_bound_trace(dk, q2=1125899906826241):
    """The FFT trace (br2f_trace; context.hip, apriori_bound level 4): 11 steps, 25 rows of the trace
    key [11][25][2 out][2048] as two 25-bit limbs, digits |d| <= 3 (balanced base 4, the top one in
    [-2, 3]), accumulated in row order."""
    r = _centred(dk.trace_key.reshape(11, 25, 2, 2048), q2)
    hi = np.rint(r / 2.0 ** 25)
    k = np.stack([_row_max(r - hi * 2.0 ** 25, 1024), _row_max(hi, 1024)], axis=-1).reshape(11, 25, 4)
    return _bound(k, 1024, 25, 3.0, list(range(25)), 41 + 26)
