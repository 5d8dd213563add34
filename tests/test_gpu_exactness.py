"""Exactness of the FFT external products at the timed geometry.

The reference computes every external product with an exact modular NTT (concrete-ntt,
omr_core/Cargo.toml:38-45; detector.rs:553-557, :623). The throughput kernels here use FP64
FFTs and round (br1_fft.hpp, br2_fft.hpp; the latency level 1 too), so these tests prove the
rounding exact on bench.py's own keys and clues (pack 42, key seed 7, clue seeds 1000 / 1001):

- the rounding-margin guard (exactness.hpp) over one 65,536-message launch: the largest
  |y - rint(y)| of every rounded coefficient of both levels is < 0.1, the guarded output equals
  the production output, and the run is certified by the a priori bound (observed < 1 - E);
- the a priori bounds the library computes from its stored key spectra equal the numpy
  restatement (tests/fft_bound.py) and are < 0.5 on both levels: exact for every input on this key;
- the same 65,536 clues through the latency family with the threshold raised, so level 2 runs
  br2l_kernel's exact modular NTT (and trace_kernel): all 65,536 outputs bit-identical to the
  throughput family's;
- the double-double key spectra: sampled rows against a long-double restatement of the same tree
  transform, |K^ - K| <= u |K| as the bound assumes, and kappa >= every sampled |K^|;
- the context's hand-off buffers across mixed call sizes: detect 8 -> level-2
  rotation of 16 -> detect 8, increasing and decreasing sizes with a raised threshold (br2x
  accepted while trace_x is refused), each bit-exact against the throughput path, and
  omr_ctx_check OK at the end.
"""
import numpy as np
import pytest

import product_lib as PL
from product_lib import omr_amd as A

pytestmark = pytest.mark.gpu
U = 2.0 ** -53
D_FULL = 65536


def _device_clues(a, b, D, mask):
    import torch
    dev = torch.device("cuda", 0)
    ca = torch.empty((D, A.N0), dtype=torch.int16, device=dev)
    cb = torch.empty((D, A.CLUE_COUNT), dtype=torch.int16, device=dev)
    na, nb = torch.empty_like(ca), torch.empty_like(cb)
    a.gen_clues_device(1000, 0, D, ca.data_ptr(), cb.data_ptr())
    b.gen_clues_device(1001, 0, D, na.data_ptr(), nb.data_ptr())
    m = torch.from_numpy(mask).to(dev)[:, None]
    return torch.where(m, ca, na).contiguous(), torch.where(m, cb, nb).contiguous()


@pytest.fixture(scope="module")
def full():
    """bench.py's D = 65,536 board: production output (one 65,536-message launch) and clues."""
    import torch
    a, b, dk = PL.keys()
    det = A.Detector(dk)
    rng = np.random.default_rng(2025)
    pert = np.sort(rng.choice(D_FULL, 50, replace=False))
    mask = np.zeros(D_FULL, dtype=bool)
    mask[pert] = True
    d_ca, d_cb = _device_clues(a, b, D_FULL, mask)
    out = torch.empty((D_FULL, 2, 2048), dtype=torch.int64, device="cuda:0")
    det.set_batch(D_FULL)
    torch.cuda.synchronize()
    det.detect_batch_device(d_ca.data_ptr(), d_cb.data_ptr(), D_FULL, out.data_ptr(), None)
    det.check()
    yield det, d_ca, d_cb, out, mask
    det.close()


def test_rounding_margin_full_launch_certified(full):
    import torch
    det, d_ca, d_cb, want, _ = full
    det.rounding_margin(reset=True)
    det.set_rounding_guard(True)
    got = torch.empty_like(want)
    det.detect_batch_device(d_ca.data_ptr(), d_cb.data_ptr(), D_FULL, got.data_ptr(), None)
    det.check()
    det.set_rounding_guard(False)
    m = det.rounding_margin(reset=True)
    assert torch.equal(got, want), "guarded kernels changed the output"
    obs, apr = m["observed"], m["apriori"]
    print(f"\nrounding margin over {D_FULL} messages: level 1 {obs[0]:.3e}, level 2 {obs[1]:.3e}; "
          f"a priori bounds {apr[0]:.3f}, {apr[1]:.3f}; kappa {m['kappa']}")
    assert 0 < obs[0] < 0.1 and 0 < obs[1] < 0.1
    # the library's bound on its stored (double-double) spectra equals the numpy restatement
    from fft_bound import apriori_bounds
    e1, e2, k1, k2 = apriori_bounds(PL.keys()[2])
    assert abs(apr[0] - e1) < 1e-9 * e1 and abs(apr[1] - e2) < 1e-9 * e2, (apr, e1, e2)
    assert abs(m["kappa"][0] - k1) < 1e-9 * k1 and abs(m["kappa"][1] - k2) < 1e-9 * k2
    assert apr[0] < 0.5 and apr[1] < 0.5, "both levels exact for every input on this key"
    for lvl in range(2):
        assert obs[lvl] < 1 - apr[lvl], f"level {lvl + 1}: run not certified"


def test_latency_family_exact_ntt_matches_full_launch(full):
    """All 65,536 outputs of the throughput family (FFT level 2) equal the latency family's, whose
    level 2 (br2l_kernel at this size: the two-CU launch does not fit) is the exact modular NTT."""
    import torch
    det, d_ca, d_cb, want, mask = full
    det.set_latency_threshold(D_FULL)
    got = torch.empty_like(want)
    try:
        det.detect_batch_device(d_ca.data_ptr(), d_cb.data_ptr(), D_FULL, got.data_ptr(), None)
        det.check()
    finally:
        det.set_latency_threshold(64)
    diff = (got != want).reshape(D_FULL, -1).any(dim=1)
    bad = torch.nonzero(diff).flatten()[:8].tolist()
    assert not bad, f"{int(diff.sum())} messages differ between the FFT and NTT level 2, e.g. {bad}"


def test_exact_level1_ntt_matches_full_launch(full):
    """All 65,536 outputs with level 1 on the exact modular NTT (omr_ctx_set_exact_level1:
    br1n_kernel, the reference's arithmetic for all 458,752 rotations) equal the production FFT
    launch's: the full-size check of the level-1 FFT that the latency family cannot give (both
    families share the level-1 FFT)."""
    import time
    import torch
    det, d_ca, d_cb, want, mask = full
    got = torch.empty_like(want)
    det.set_exact_level1(True)
    try:
        t = time.perf_counter()
        det.detect_batch_device(d_ca.data_ptr(), d_cb.data_ptr(), D_FULL, got.data_ptr(), None)
        det.check()
        print(f"\nexact-NTT level 1 + FFT level 2 over {D_FULL} messages: {time.perf_counter() - t:.2f} s")
    finally:
        det.set_exact_level1(False)
    diff = (got != want).reshape(D_FULL, -1).any(dim=1)
    bad = torch.nonzero(diff).flatten()[:8].tolist()
    assert not bad, f"{int(diff.sum())} messages differ between the FFT and NTT level 1, e.g. {bad}"


# ---- double-double key spectra ------------------------------------------------------------------
def _tree_fft_ld(z, L):
    """The natural-order tree transform of key_spectra.hpp in numpy long double (64-bit mantissa)."""
    n = 1 << L
    pi = np.arctan(np.longdouble(1)) * 4
    x = z.astype(np.clongdouble).copy()
    eps = [n]
    for s in range(L):
        lh = L - 1 - s
        h = 1 << lh
        half = np.array([e // 2 for e in eps], dtype=np.int64)
        ang = pi * np.array(half % (4 * n), dtype=np.longdouble) / np.longdouble(2 * n)
        w = np.cos(ang) + 1j * np.sin(ang)
        xv = x.reshape(x.shape[0], 1 << s, 2, h)
        v = w[None, :, None] * xv[:, :, 1, :]
        a, b = xv[:, :, 0, :] + v, xv[:, :, 0, :] - v
        xv[:, :, 0, :], xv[:, :, 1, :] = a, b
        eps = [y for e in eps for y in ((e // 2) % (4 * n), (e // 2 + 2 * n) % (4 * n))]
    return x


def _jidx3(lane, e):  # device_fft.hpp WgFft::jidx(3, lane, e)
    l5 = (lane >> 5) & 1
    return ((lane & 31) << 4) | (l5 << 3) | (((e >> 1) & 1) << 2) | ((e & 1) << 1) | ((e >> 2) & 1)


def _centred(v, q):
    v = v.astype(np.int64) if q < 2 ** 62 else v
    return np.where(v > (q - 1) // 2, v.astype(np.float64) - q, v.astype(np.float64))


@pytest.mark.parametrize("level", [1, 2])
def test_key_spectra_double_double(level):
    import fft2_model as M2
    _, _, dk = PL.keys()
    det = A.Detector(dk)
    kappa = det.rounding_margin()["kappa"][level - 1]
    if level == 1:
        rows = dk.bsk1.reshape(-1, 1024)
        picks = [0, 1, 2, 3, 4095, 8191]
        n, L = 512, 9
        slot_index = np.array([_jidx3(s & 63, s >> 6) for s in range(n)])
        per = 1
    else:
        rows = dk.bsk2.reshape(-1, 2048)
        picks = [0, 5, 6, 11, 8000, 16079]
        n, L = 1024, 10
        slot_index = np.array([M2.idx(4, s & 255, s >> 8) for s in range(n)])
        per = 2
    worst, kmax = 0.0, 0.0
    for p in picks:
        got = det.key_spectrum(level, p * per * n, per * n).reshape(per, n)
        c = _centred(rows[p], A.Q1 if level == 1 else A.Q2)
        if level == 1:
            limbs = [c]
        else:
            hi = np.rint(c / 2.0 ** 25)
            limbs = [c - hi * 2.0 ** 25, hi]
        for lb, cl in enumerate(limbs):
            z = (cl[:n] + 1j * cl[n:])[None, :]
            K = (_tree_fft_ld(z, L)[0] / n)[slot_index]
            err = np.abs(got[lb].astype(np.clongdouble) - K)
            assert np.all(err <= U * np.abs(K) * (1 + 2 ** -10) + 1e-18 * kappa), f"row {p} limb {lb}"
            worst = max(worst, float(np.max(err / np.maximum(np.abs(K), 1e-300))))
            kmax = max(kmax, float(np.max(np.abs(got[lb]))))
    det.close()
    assert kmax <= kappa * (1 + 1e-12)
    print(f"\nlevel {level}: worst |K^ - K| / |K| = {worst / U:.3f} u over the sampled rows; kappa {kappa:.4e}")


# ---- hand-off buffers across mixed call sizes --------------------------------------
def test_handoff_buffers_mixed_sizes():
    a, b, dk = PL.keys()
    det = A.Detector(dk)
    ref = A.Detector(dk)
    ref.set_latency_threshold(0)  # throughput kernels only
    num_cu = 256

    def lwes(n, seed):
        rng = np.random.default_rng(seed)
        x = rng.integers(0, 4096, size=(n, A.NI + 1), dtype=np.uint32)
        return x

    def check_detect(n, seed):
        mask = np.arange(n) % 5 == 0
        ca, cb = PL.mixed_clues(mask, seed=seed)
        assert np.array_equal(det.detect_batch(ca, cb), ref.detect_batch(ca, cb)), f"detect {n}"

    def check_level2(n, seed):
        x = lwes(n, seed)
        assert np.array_equal(det.blind_rotate_level2(x), ref.blind_rotate_level2(x)), f"level 2 {n}"

    check_detect(8, 1)
    check_level2(16, 2)   # grows the two-CU slots only
    check_detect(8, 3)    # the trace slots of the first call must still be valid
    det.set_latency_threshold(num_cu)  # n in (0.4, 0.5] x num_cu: br2x accepted, trace_x refused
    for n, s in ((110, 4), (128, 5), (40, 6), (8, 7)):
        check_detect(n, s)
    check_level2(100, 8)
    check_detect(8, 9)
    det.check()
    det.close()
    ref.close()


# ---- the exactness contract -----------------------------------------------
def test_high_kappa_key_guarded_and_oracle_exact():
    """A key whose a priori bound E2 is >= 1 (tests/crafted_keys.py: aligned maximal level-2 limbs on
    four steps): the context guards level 2 on every launch without being asked, every such launch
    breaches the threshold 1 - E2 <= 0 and is re-run on the exact NTT (br2l_fallback_kernel +
    trace_fallback_kernel), and the outputs equal the oracle's -- fused trace (timing off) and the
    split trace (detect_with_time_info) alike, and the level-2 stage entry."""
    import crafted_keys as CK
    import oracle_lib as O
    _, _, dk = PL.keys()
    ck = A.DetectionKey(dk.bsk1, dk.ksk, CK.high_kappa_bsk2(dk.bsk2), dk.trace_key)
    det = A.Detector(ck)
    try:
        m = det.rounding_margin()
        assert m["apriori"][0] < 0.5 <= 1.0 <= m["apriori"][1], m
        from fft_bound import apriori_bounds
        e1, e2, _, _ = apriori_bounds(ck)
        assert abs(m["apriori"][1] - e2) < 1e-9 * e2
        ex = det.exactness()
        assert ex == {"guarded": [False, True], "breaches": [0, 0]}, ex
        det.set_latency_threshold(0)  # throughput kernels: the FFT level 2
        mask = np.arange(72) % 9 == 0
        ca, cb = PL.mixed_clues(mask, seed=77)
        got = det.detect_batch(ca, cb)
        ex = det.exactness()
        assert ex["guarded"] == [False, True] and ex["breaches"][0] == 0 and ex["breaches"][1] >= 1, ex
        got_split, _ = det.detect_with_time_info(ca[:40], cb[:40])
        assert det.exactness()["breaches"][1] > ex["breaches"][1]
        orc = O.OracleDetector(ck.bsk1, ck.ksk, ck.bsk2, ck.trace_key)
        try:
            ref = orc.detect_batch(ca, cb)
            lwe = np.stack([orc.first_level(ca[i], cb[i]) for i in range(8)])
            ref_rot = np.stack([orc.br2(x) for x in lwe])
        finally:
            orc.close()
        assert np.array_equal(got, ref), "guarded high-kappa detect differs from the oracle"
        assert np.array_equal(got_split, ref[:40]), "split-trace path differs from the oracle"
        assert np.array_equal(det.blind_rotate_level2(lwe), ref_rot), "level-2 rotation entry differs"
        det.check()
    finally:
        det.close()


def test_high_kappa_level1_key_rerun_exact():
    """A key whose level-1 a priori bound E1 is >= 1 (tests/crafted_keys.py: aligned maximal BSK1
    rows on four steps): the context guards level 1 on every launch without being asked, every such
    launch breaches the threshold 1 - E1 <= 0 and is re-run on the exact NTT (br1n_fallback_kernel),
    and the outputs equal the oracle's on both kernel families and through the level-1 entries."""
    import crafted_keys as CK
    import oracle_lib as O
    _, _, dk = PL.keys()
    ck = A.DetectionKey(CK.high_kappa_bsk1(dk.bsk1), dk.ksk, dk.bsk2, dk.trace_key)
    det = A.Detector(ck)
    try:
        m = det.rounding_margin()
        assert m["apriori"][1] < 0.5 <= 1.0 <= m["apriori"][0], m
        from fft_bound import apriori_bounds
        e1, _, _, _ = apriori_bounds(ck)
        assert abs(m["apriori"][0] - e1) < 1e-9 * e1
        assert det.exactness() == {"guarded": [True, False], "breaches": [0, 0]}
        mask = np.arange(72) % 9 == 0
        ca, cb = PL.mixed_clues(mask, seed=78)
        det.set_latency_threshold(0)  # throughput kernels: br1f_guard_kernel + the fallback
        got = det.detect_batch(ca, cb)
        ex = det.exactness()
        assert ex["guarded"] == [True, False] and ex["breaches"][0] >= 1 and ex["breaches"][1] == 0, ex
        det.set_latency_threshold(64)  # latency kernels: br1l_guard_kernel + the fallback
        got_lat = det.detect_batch(ca[:5], cb[:5])
        assert det.exactness()["breaches"][0] > ex["breaches"][0]
        orc = O.OracleDetector(ck.bsk1, ck.ksk, ck.bsk2, ck.trace_key)
        try:
            ref = orc.detect_batch(ca, cb)
            lwe = np.stack([orc.first_level(ca[i], cb[i]) for i in range(3)])
        finally:
            orc.close()
        assert np.array_equal(got, ref), "guarded high-kappa level-1 detect differs from the oracle"
        assert np.array_equal(got_lat, ref[:5]), "latency family differs from the oracle"
        assert np.array_equal(det.first_level(ca[:3], cb[:3]), lwe), "level-1 stage entry differs"
        det.check()
    finally:
        det.close()


def test_exact_level1_small_matches_oracle():
    """omr_ctx_set_exact_level1 at oracle sizes: both detect families and the mode-1 rotation entry
    (explicit LWEs -> full RLWE) equal the oracle with level 1 on br1n_kernel."""
    import oracle_lib as O
    _, _, dk = PL.keys()
    det = A.Detector(dk)
    try:
        det.set_exact_level1(True)
        mask = np.arange(70) % 7 == 0
        ca, cb = PL.mixed_clues(mask, seed=79)
        det.set_latency_threshold(0)
        got = det.detect_batch(ca, cb)
        det.set_latency_threshold(64)
        got_lat = det.detect_batch(ca[:3], cb[:3])
        rng = np.random.default_rng(80)
        la = rng.integers(0, 2048, size=(5, 512), dtype=np.uint16)
        lb = rng.integers(0, 2048, size=5, dtype=np.uint16)
        rot = det.blind_rotate_level1(la, lb)
        det.set_exact_level1(False)
        assert np.array_equal(det.blind_rotate_level1(la, lb), rot), "FFT vs NTT level-1 rotation entry"
        orc = O.OracleDetector(dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key)
        try:
            ref = orc.detect_batch(ca, cb)
        finally:
            orc.close()
        assert np.array_equal(got, ref), "exact-NTT level 1 (throughput family) differs from the oracle"
        assert np.array_equal(got_lat, ref[:3]), "exact-NTT level 1 (latency family) differs from the oracle"
        det.check()
    finally:
        det.close()


@pytest.mark.parametrize("pack_seed,key_seed", [(42, 8), (43, 7), (4242, 11)])
def test_apriori_bound_below_half_on_gpu_generated_keys(pack_seed, key_seed):
    """Three more GPU-generated keys: both bounds below 0.5, so no launch needs the guard."""
    import torch
    dev = torch.device("cuda", 0)
    pack = A.SecretKeyPack(pack_seed)
    bufs = [torch.empty(int(np.prod(shape)), dtype=dt, device=dev)
            for shape, dt in ((A.BSK1_SHAPE, torch.int32), (A.KSK_SHAPE, torch.int32),
                              (A.BSK2_SHAPE, torch.int64), (A.TK_SHAPE, torch.int64))]
    pack.generate_detection_key_device(key_seed, *[b.data_ptr() for b in bufs])
    det = A.Detector.from_device_key(*[b.data_ptr() for b in bufs])
    try:
        apr = det.rounding_margin()["apriori"]
        print(f"\npack {pack_seed} key {key_seed}: E1 {apr[0]:.4f}, E2 {apr[1]:.4f}")
        assert apr[0] < 0.5 and apr[1] < 0.5, apr
        assert det.exactness() == {"guarded": [False, False], "breaches": [0, 0]}
    finally:
        det.close()


def test_apriori_bound_margin_over_16_gpu_keys():
    """The exactness margin over 16 GPU-generated keys (E2 rose to 0.445 with the
    tangent-form forward transforms, 0.055 below the threshold at which a context guards level 2 on
    every launch). Reports every key's E1 / E2 and the maxima; every key must stay below 0.5 (else
    its context would be guarded automatically: still exact, but on the guarded kernels)."""
    import torch
    dev = torch.device("cuda", 0)
    rows = []
    for i in range(16):
        pack_seed, key_seed = 1000 + 37 * i, 11 + i
        pack = A.SecretKeyPack(pack_seed)
        bufs = [torch.empty(int(np.prod(shape)), dtype=dt, device=dev)
                for shape, dt in ((A.BSK1_SHAPE, torch.int32), (A.KSK_SHAPE, torch.int32),
                                  (A.BSK2_SHAPE, torch.int64), (A.TK_SHAPE, torch.int64))]
        pack.generate_detection_key_device(key_seed, *[b.data_ptr() for b in bufs])
        det = A.Detector.from_device_key(*[b.data_ptr() for b in bufs])
        try:
            rm = det.rounding_margin()
            rows.append((pack_seed, key_seed, rm["apriori"][0], rm["apriori"][1], rm["kappa"][0], rm["kappa"][1],
                         det.exactness()["guarded"]))
        finally:
            det.close()
        del bufs
    print("\npack  key   E1      E2      kappa1     kappa2     guarded")
    for r in rows:
        print(f"{r[0]:5d} {r[1]:4d}  {r[2]:.4f}  {r[3]:.4f}  {r[4]:.4e} {r[5]:.4e} {r[6]}")
    e1, e2 = max(r[2] for r in rows), max(r[3] for r in rows)
    print(f"max E1 {e1:.4f}, max E2 {e2:.4f} over {len(rows)} keys (margin to 0.5: {0.5 - e2:.4f})")
    assert e1 < 0.5 and e2 < 0.5, (e1, e2)
    assert all(r[6] == [False, False] for r in rows)
