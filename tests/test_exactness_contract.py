"""The exactness contract on the CPU side.

The reference's external products are exact for every key (concrete-ntt, omr_core/Cargo.toml:38-45;
detector.rs:553-557, :623). The product's FFT products are exact whenever the key's a priori bound E
 is below 0.5; a key with E >= 0.5 switches the context to guarded kernels on every
launch (context.hip, omr_ctx_exactness). Here: the numpy restatement of E (tests/fft_bound.py) on a
uniform key is below 0.5 on both levels, and the crafted high-kappa key of tests/crafted_keys.py
(aligned maximal level-2 limbs on four steps) puts E2 above 1, so a context built from it must
guard level 2 (checked on the GPU in tests/test_gpu_exactness.py). The ABI declares the status
and the query the contract adds."""
import os
import types

import numpy as np

import crafted_keys as CK
import fft_bound as FB

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
Q1 = 134215681


def _uniform_key(seed=5):
    rng = np.random.default_rng(seed)
    bsk1 = rng.integers(0, Q1, size=(512, 8, 2, 1024), dtype=np.uint64).astype(np.uint32)
    bsk2 = rng.integers(0, CK.Q2, size=(670, 12, 2, 2048), dtype=np.uint64)
    return types.SimpleNamespace(bsk1=bsk1, bsk2=bsk2)


def test_apriori_bound_uniform_key_below_half_and_crafted_key_above():
    dk = _uniform_key()
    e1, e2, k1, k2 = FB.apriori_bounds(dk)
    assert e1 < 0.5 and e2 < 0.5, (e1, e2)
    crafted = types.SimpleNamespace(bsk1=dk.bsk1, bsk2=CK.high_kappa_bsk2(dk.bsk2))
    c1, c2, ck1, ck2 = FB.apriori_bounds(crafted)
    assert c1 == e1 and ck1 == k1, "level 1 untouched"
    assert ck2 > 10 * k2, (ck2, k2)
    assert c2 >= 1.0, f"crafted key E2 = {c2}: the guard must be on and every launch re-run exactly"
    # the crafted limb peak: 4 / pi of the limb bound (sum of |cos| + |sin| over the quarter turn)
    assert abs(ck2 / CK.LIMB_MAX - 4 / np.pi) < 1e-3
    crafted1 = types.SimpleNamespace(bsk1=CK.high_kappa_bsk1(dk.bsk1), bsk2=dk.bsk2)
    d1, d2, dk1, dk2 = FB.apriori_bounds(crafted1)
    assert d2 == e2 and dk2 == k2, "level 2 untouched"
    assert dk1 > 5 * k1 and d1 >= 1.0, (d1, dk1, k1)


def test_header_declares_the_contract():
    hdr = open(os.path.join(ROOT, "include", "omr_gpu.h")).read()
    assert "OMR_ERR_INEXACT" not in hdr  # level-1 breaches are re-run exactly, never reported
    assert "omr_status omr_ctx_exactness(omr_ctx *ctx, int guarded[2], uint64_t breaches[2]);" in hdr


def test_trace_fft_bound_far_below_level2():
    """The FFT trace's a priori bound (digits |d| <= 3 over 25 rows) on a uniform key: far below 0.5
    and below level 2's, so trace_fft_kernel runs on every real key (context.hip: trace_fft)."""
    dk = _uniform_key()
    rng = np.random.default_rng(9)
    dk.trace_key = rng.integers(0, CK.Q2, size=(11, 25, 2, 2048), dtype=np.uint64)
    et = FB.apriori_bound_trace(dk)
    _, e2, _, _ = FB.apriori_bounds(dk)
    assert 0 < et < 0.5 and et < e2, (et, e2)
