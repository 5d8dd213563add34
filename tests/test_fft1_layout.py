"""Level-1 FFT layout (tfhe-omr_amd/csrc/device_fft.hpp, WgFft::jidx / slot, restated here): the
four pass layouts are bijections, the permlane swaps (register bits 2, 1 <-> lane bits 5, 4 after
pass 0; register bit 2 <-> lane bit 5 after pass 2) produce the next pass's layout, the one LDS
exchange is bank-conflict free in both directions, and the numpy models of the kernel's pass
structure (tools/fft_exactness.py: Fft8P, the premultiplied passes of rounds 2-4; Fft8PT, the
tangent-form forward butterflies of round 5) return the exact negacyclic product after rounding,
and agree with each other to rounding."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import fft_exactness as FX  # noqa: E402

LANE = np.arange(64)


def jidx(p, lane, e):
    l5, l4 = (lane >> 5) & 1, (lane >> 4) & 1
    if p == 0:
        return (e << 6) | lane
    if p == 1:
        return (l5 << 8) | (l4 << 7) | ((e & 1) << 6) | (((e >> 2) & 1) << 5) | (((e >> 1) & 1) << 4) | (lane & 15)
    if p == 2:
        return ((lane & 31) << 4) | (e << 1) | l5
    return ((lane & 31) << 4) | (l5 << 3) | (((e >> 1) & 1) << 2) | ((e & 1) << 1) | ((e >> 2) & 1)


def slot(j):
    return j ^ ((j >> 4) & 1) ^ (((j >> 5) & 1) << 1) ^ (((j >> 6) & 1) << 2) ^ (((j >> 8) & 1) << 3)


def apply_swaps(p_from, lane, e, swaps):
    """index now at (lane, e) after swapping register bit rb with lane bit lb for each (rb, lb)"""
    st, se = lane, e
    for rb, lb in swaps:
        lt, le = (st >> lb) & 1, (se >> rb) & 1
        st = (st & ~(1 << lb)) | (le << lb)
        se = (se & ~(1 << rb)) | (lt << rb)
    return jidx(p_from, st, se)


def test_layouts_bijective():
    for p in range(4):
        idx = np.concatenate([jidx(p, LANE, e) for e in range(8)])
        assert np.array_equal(np.sort(idx), np.arange(512))
    assert np.array_equal(jidx(0, LANE, 3), LANE + 64 * 3)  # coefficient layout lane + 64 e


def test_permlane_relayouts():
    for lane in range(64):
        for e in range(8):
            assert apply_swaps(0, lane, e, [(2, 5), (1, 4)]) == jidx(1, lane, e)
            assert apply_swaps(2, lane, e, [(2, 5)]) == jidx(3, lane, e)


def test_exchange_conflict_free():
    assert np.array_equal(np.sort(slot(np.arange(512))), np.arange(512))
    # MI355X_MICROARCH.md LDS table: ds_write_b128 8 groups of 8 contiguous lanes (16-B slot mod 8
    # distinct), ds_read_b128 4 groups of 16 lanes (slot mod 16 distinct)
    g16 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
           list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
    g16 += [[x + 32 for x in g] for g in g16]
    for pw, pr in ((1, 2), (2, 1)):
        for e in range(8):
            w, r = slot(jidx(pw, LANE, e)), slot(jidx(pr, LANE, e))
            for g in range(0, 64, 8):
                assert len(set((w[g:g + 8] % 8).tolist())) == 8
            for g in g16:
                assert len(set((r[g] % 16).tolist())) == 16


@pytest.mark.parametrize("model", ["Fft8P", "Fft8PT"])
def test_model_exact_product(model):
    f = getattr(FX, model)()
    for lane_e in [(p, e) for p in range(4) for e in range(8)]:
        assert np.array_equal(f.jidx(*lane_e), jidx(lane_e[0], LANE, lane_e[1]))
    rng = np.random.default_rng(3)
    N = 1024
    keys = [rng.integers(-(1 << 26), 1 << 26, N) for _ in range(8)]
    for digs in ([rng.integers(-17, 18, N) for _ in range(8)], FX.adversarial(keys, 17, N, rng)):
        exact = np.array(sum(FX.negacyclic(d, k) for d, k in zip(digs, keys)), dtype=np.float64)
        acc = sum(f.fwd(FX.fold(d.astype(float))) * (f.fwd(FX.fold(k.astype(float))) / 512)
                  for d, k in zip(digs, keys))
        out = FX.unfold(f.inv(acc))
        assert np.array_equal(np.rint(out), exact)
        assert np.max(np.abs(out - exact)) < 0.01


def test_tangent_model_matches_premultiplied():
    rng = np.random.default_rng(11)
    z = rng.standard_normal(512) + 1j * rng.standard_normal(512)
    a, b = FX.Fft8P(), FX.Fft8PT()
    fa, fb = a.fwd(z), b.fwd(z)
    assert np.max(np.abs(fa - fb)) < 1e-12 * np.max(np.abs(fa))
    assert np.max(np.abs(b.inv(fb) / 512 - z)) < 1e-12
