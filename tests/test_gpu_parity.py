"""GPU parity: every HIP stage through the C ABI against the oracle / golden vectors, bit-exact."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import product_lib as PL
import retriever as R
from product_lib import omr_amd as A

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(PL.ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def prim():
    with open(os.path.join(GOLDEN, "primitives.json")) as f:
        return json.load(f)


def _negacyclic_mod_q1(d, k):
    """Exact d * k mod (X^1024 + 1, q1) (int64 is exact: |d| <= 17, |k| < 2^27, 1024 terms)."""
    full = np.convolve(d.astype(np.int64), k.astype(np.int64))
    r = full[:1024].copy()
    r[:1023] -= full[1024:]
    return (r % A.Q1).astype(np.uint64)


def test_gpu_fft1_product_exact():
    """The level-1 FFT external product (device_fft.hpp) returns the exact integer product for
    digit-sized inputs: random digits, and digits of maximal magnitude aligned with the key's
    signs for one output coefficient (the worst case for rounding error)."""
    a_sk, _, dk = PL.keys()
    det = A.Detector(dk)
    rng = np.random.default_rng(11)
    q1 = A.Q1
    keys = rng.integers(-(q1 - 1) // 2, (q1 - 1) // 2 + 1, (6, 1024))
    digs = [rng.integers(-17, 18, 1024) for _ in range(3)]
    for c in (0, 511, 1023):  # out_c = sum_j d_j * k_{c-j} (negated when wrapped)
        k = keys[len(digs)]
        t = (c - np.arange(1024)) % 1024
        sign = np.where(np.arange(1024) <= c, 1, -1)
        digs.append(17 * sign * np.sign(k[t]).astype(np.int64))
    got = det.fft1_mul(np.stack([d % q1 for d in digs]).astype(np.uint32), (keys % q1).astype(np.uint32))
    for i, d in enumerate(digs):
        assert np.array_equal(got[i], _negacyclic_mod_q1(d, keys[i])), f"case {i}"


@pytest.mark.parametrize("level", [1, 2])
def test_gpu_ntt_matches_definition(prim, level):
    vecs = prim["ntt"][str(level)]
    inp = np.array([v["in"] for v in vecs], dtype=np.uint64)
    out = A.ntt(level, inp)
    assert out.tolist() == [v["out"] for v in vecs]
    back = A.ntt(level, out, inverse=True)
    assert np.array_equal(back, inp)
    # random batch vs oracle
    q = A.Q1 if level == 1 else A.Q2
    n = 1024 if level == 1 else 2048
    rnd = np.random.default_rng(level).integers(0, q, (64, n), dtype=np.uint64)
    g = A.ntt(level, rnd)
    for k in range(0, 64, 9):
        assert np.array_equal(g[k], O.ntt(level, rnd[k]))
    assert np.array_equal(A.ntt(level, g, inverse=True), rnd)


@pytest.fixture(scope="module")
def structured():
    import structured_keys
    keys, expect = structured_keys.load()
    dk = A.DetectionKey(keys["bsk1"], keys["ksk"], keys["bsk2"], keys["tk"])
    det = A.Detector(dk)
    yield det, expect
    det.close()


@pytest.mark.parametrize("threshold", [64, 0])
def test_structured_stages(structured, threshold):
    """Every stage on structured keys against the independent model's golden vectors, through the
    latency kernels (threshold 64) and the throughput kernels (threshold 0)."""
    det, e = structured
    det.set_latency_threshold(threshold)
    try:
        la = np.zeros(512, dtype=np.uint16)
        lb = np.zeros(1, dtype=np.uint16)
        O.lib().oref_extract_clue(e["clue_a"], e["clue_b"], 0, la, lb)
        assert np.array_equal(det.blind_rotate_level1(la, lb)[0], e["br1_clue0"])
        assert np.array_equal(det.first_level(e["clue_a"], e["clue_b"])[0], e["lwe_int"])
        assert np.array_equal(det.blind_rotate_level2(e["lwe_int"])[0], e["br2"])
        assert np.array_equal(det.second_level(e["lwe_int"])[0], e["detect"])
        assert np.array_equal(det.detect(e["clue_a"], e["clue_b"]), e["detect"])
    finally:
        det.set_latency_threshold(64)


@pytest.fixture(scope="module")
def real():
    a, b, dk = PL.keys()
    det = A.Detector(dk)
    orc = O.OracleDetector(dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key)
    yield a, det, orc
    det.close()
    orc.close()


@pytest.fixture(params=["latency", "throughput"])
def path(request, real):
    """Both kernel families on the same small inputs: the latency kernels (chunks up to 64
    messages by default, latency_kernels.hpp) and the throughput kernels (threshold 0)."""
    det = real[1]
    det.set_latency_threshold(64 if request.param == "latency" else 0)
    yield request.param
    det.set_latency_threshold(64)


def test_real_keys_detect_bit_exact_and_kat(real, path):
    a, det, orc = real
    s2 = a.export()["s2"]
    mask = np.array([1, 0, 1, 0, 0, 1, 0, 1], dtype=bool)
    ca, cb = PL.mixed_clues(mask, seed=31)
    gpu = det.detect_batch(ca, cb)
    ref = orc.detect_batch(ca, cb)
    assert np.array_equal(gpu, ref)
    for m in range(len(mask)):
        dec = R.decrypt_decode(s2, gpu[m])
        if mask[m]:
            assert dec[0] == 1 and not dec[1:].any()
        else:
            assert not dec.any()


def test_real_keys_stage_parity(real, path):
    _, det, orc = real
    ca, cb = PL.mixed_clues([True, False, False], seed=7)
    fl = det.first_level(ca, cb)
    for m in range(3):
        assert np.array_equal(fl[m], orc.first_level(ca[m], cb[m]))
    br = det.blind_rotate_level2(fl[:1])
    assert np.array_equal(br[0], orc.br2(fl[0]))
    assert np.array_equal(det.second_level(fl[:1])[0], orc.trace(br[0]))


def test_latency_level2_variants_match_throughput(real):
    """The latency path's level 2 in both forms against the (oracle-checked) throughput kernels,
    bit for bit: the two-CU kernel (br2y, the default; br2x is checked against it in
    test_latency_level2_fft_two_cu_matches_ntt) at 64 messages (128 workgroups, the default
    threshold's largest chunk) and the one-CU kernel br2l, which runs when 2 n workgroups exceed the
    CU count (130 messages with the threshold raised); every output passes the omd KAT."""
    a, det, _ = real
    s2 = a.export()["s2"]
    for n, threshold in ((64, 64), (130, 200)):
        mask = np.zeros(n, dtype=bool)
        mask[::9] = True
        ca, cb = PL.mixed_clues(mask, seed=900 + n)
        det.set_latency_threshold(threshold)
        try:
            lat = det.detect_batch(ca, cb)
        finally:
            det.set_latency_threshold(0)
        thr = det.detect_batch(ca, cb)
        det.set_latency_threshold(64)
        assert np.array_equal(lat, thr)
        for m in range(n):
            dec = R.decrypt_decode(s2, lat[m])
            assert (dec[0] == 1) == mask[m] and not dec[1:].any()


def test_latency_level2_fft_two_cu_matches_ntt(real, monkeypatch):
    """The latency path's level 2 on the FFT over two CUs per message (br2y_kernel, the default: it
    runs when the a priori bound of its accumulation order is below 0.5) against the exact
    modular-NTT two-CU kernel (br2x_kernel: a context created with OMR_BR2Y=0) on the same level-1
    outputs, bit for bit, rotation and rotation + trace, at 1, 7, 20 and 64 messages (2, 14, 40 and
    128 CUs; the first three with four key-prefetch helper workgroups per worker, 64 without), and
    at 7 br2y without its helpers (OMR_PREFETCH=0) and with the sc1 hand-off kept between workers
    on one XCD (OMR_FAST_HANDOFF=0: the other side of its placement-dependent protocol choice)."""
    _, fft, _ = real
    _, _, dk = PL.keys()
    monkeypatch.setenv("OMR_BR2Y", "0")
    ntt = A.Detector(dk)
    monkeypatch.delenv("OMR_BR2Y")
    monkeypatch.setenv("OMR_PREFETCH", "0")
    nopf = A.Detector(dk)
    monkeypatch.delenv("OMR_PREFETCH")
    monkeypatch.setenv("OMR_FAST_HANDOFF", "0")
    slow = A.Detector(dk)
    monkeypatch.delenv("OMR_FAST_HANDOFF")
    try:
        for n in (1, 7, 20, 64):
            mask = np.zeros(n, dtype=bool)
            mask[::5] = True
            ca, cb = PL.mixed_clues(mask, seed=1200 + n)
            fl = fft.first_level(ca, cb)
            want = ntt.blind_rotate_level2(fl)
            assert np.array_equal(fft.blind_rotate_level2(fl), want), n
            assert np.array_equal(fft.second_level(fl), ntt.second_level(fl)), n
            if n == 7:
                assert np.array_equal(nopf.blind_rotate_level2(fl), want)
                assert np.array_equal(slow.blind_rotate_level2(fl), want)
    finally:
        ntt.close()
        nopf.close()
        slow.close()


def test_level2_throughput_small_batches(real):
    """The throughput level-2 kernel (br2f_kernel, FFT) at batches of 5 and 6 messages against the
    latency kernels (the oracle-checked NTT path), rotation and rotation + trace."""
    _, det, _ = real
    for n in (5, 6):
        mask = np.zeros(n, dtype=bool)
        mask[1::3] = True
        ca, cb = PL.mixed_clues(mask, seed=700 + n)
        fl = det.first_level(ca, cb)
        det.set_latency_threshold(0)
        try:
            thr_br, thr_tr = det.blind_rotate_level2(fl), det.second_level(fl)
        finally:
            det.set_latency_threshold(64)
        assert np.array_equal(thr_br, det.blind_rotate_level2(fl))
        assert np.array_equal(thr_tr, det.second_level(fl))


def test_encode_golden(structured):
    det, _ = structured
    z = np.load(os.path.join(GOLDEN, "encode.npz"))
    pv = z["pv"]
    all_count = int(z["all_count"])
    rp = A.RetrievalParams(all_count, 0)
    for k, ct in enumerate(z["idx_cts"]):
        got = det.encode_pertinent_indices(rp, pv, int(z["seed"]), int(ct), global_offset=int(z["offset"]))
        assert np.array_equal(got, z["idx"][k])
    n_ct, per_ct = int(z["n_ct"]), int(z["per_ct"])
    w, _ = O.payload_weights(z["wseed"].tobytes(), n_ct * per_ct * all_count)
    rp.cmb_cipher_count, rp.cmb_count_per_cipher = n_ct, per_ct
    got = det.encode_pertinent_payloads(pv, z["payloads"], w, rp, global_offset=int(z["offset"]))
    assert np.array_equal(got, z["pay"])


def test_batch_1024_kat_and_sampled_parity(real):
    """Config 2 size (1024 clues): every output decrypts correctly; sampled messages bit-exact."""
    a, det, orc = real
    s2 = a.export()["s2"]
    D = 1024
    rng = np.random.default_rng(3)
    mask = np.zeros(D, dtype=bool)
    mask[rng.choice(D, 50, replace=False)] = True
    ca, cb = PL.mixed_clues(mask, seed=2024)
    det.set_batch(512)  # exercise the chunk loop
    out = det.detect_batch(ca, cb)
    det.set_batch(0)
    for m in range(D):
        dec = R.decrypt_decode(s2, out[m])
        assert (dec[0] == 1) == mask[m]
        assert not dec[1:].any()
    for m in (0, 511, 512, int(np.nonzero(mask)[0][0])):
        assert np.array_equal(out[m], orc.detect(ca[m], cb[m]))


def test_end_to_end_gpu_retrieval(real):
    a, det, orc = real
    s2 = a.export()["s2"]
    D = 300
    rng = np.random.default_rng(8)
    mask = np.zeros(D, dtype=bool)
    mask[rng.choice(D, 12, replace=False)] = True
    ca, cb = PL.mixed_clues(mask, seed=555)
    pv = det.detect_batch(ca, cb)
    payloads = rng.integers(0, 256, (D, 612)).astype(np.uint16)
    rp = A.RetrievalParams(D, int(mask.sum()))
    idx = [det.encode_pertinent_indices(rp, pv, 9, ct) for ct in range(rp.max_encode_indices_cipher_count)]
    assert np.array_equal(idx[0], O.encode_indices(pv, 0, D, 9, 0))
    found = R.decode_indices(s2, idx, vars(rp), int(mask.sum()))
    assert found == set(np.nonzero(mask)[0].tolist())
    w = A.payload_weights(bytes(range(1, 33)), rp)
    pay = det.encode_pertinent_payloads(pv, payloads, w, rp)
    assert np.array_equal(pay[:2], O.encode_payloads(pv, payloads, 0, D, w, 2, 2))
    solved = R.decode_payloads(s2, pay, w, D, sorted(found), rp.combination_count)
    for i, p in zip(sorted(found), solved):
        assert p == payloads[i].tolist()


@pytest.mark.parametrize("D,layout", [
    (200, "3 index ct, 28 payload ct (55 combinations)"),
    # configs[0]: `omr --payload-count 1` — one pertinent message, 1 index digit, 7 segments per
    # ciphertext, 3 index and 3 payload ciphertexts of 6 combinations (README.md:91-93)
    (1, "3 index ct, 3 payload ct (6 combinations)"),
])
def test_native_driver_end_to_end(D, layout):
    """The C++ driver (tfhe-omr_amd/examples/omr_e2e.cpp, examples/omr.rs over the C ABI):
    detect on the GPU, encode both digests, retrieve and check indices and payloads."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(PL.ROOT, "tfhe-omr_amd"), "examples"], check=True)
    exe = os.path.join(PL.ROOT, "tfhe-omr_amd", "build", "omr_e2e")
    r = subprocess.run([exe, "-p", str(D)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"retrieval params: {layout}" in r.stdout, r.stdout
    assert f"All done: {min(D, 50)} pertinent indices and payloads recovered" in r.stdout, r.stdout


def _dev_u(n, itemsize):
    import torch
    return torch.empty(n, dtype={2: torch.int16, 4: torch.int32, 8: torch.int64}[itemsize], device="cuda:0")


def _host(t, dtype):
    return t.cpu().numpy().view(dtype)


def test_gpu_clue_generation_matches_oracle():
    """omr_gen_clues_device == the oracle's ClueKey::gen_clues restatement
    (oracle/omr_oracle_keygen.c, clue.rs:27-34) and the host generator, bit for bit, for both
    packs, at an offset global index (stream id = global message index)."""
    a_sk, b_sk, _ = PL.keys()
    for sk, pseed, seed, first, count in ((a_sk, PL.SK_SEED, 1000, 0, 257), (b_sk, PL.SK2_SEED, 1001, 123456, 1000)):
        oa, ob = O.SecretPack.generate(pseed).gen_clues(seed, first, count)
        da, db = _dev_u(count * A.N0, 2), _dev_u(count * A.CLUE_COUNT, 2)
        sk.gen_clues_device(seed, first, count, da.data_ptr(), db.data_ptr())
        assert np.array_equal(_host(da, np.uint16).reshape(oa.shape), oa)
        assert np.array_equal(_host(db, np.uint16).reshape(ob.shape), ob)
        ha, hb = sk.gen_clues(seed, first, count)
        assert np.array_equal(ha, oa) and np.array_equal(hb, ob)


def test_gpu_keygen_matches_oracle_and_detects():
    """omr_keygen_detection_key_device == the oracle's generate_detection_key
    restatement (oracle/omr_oracle_keygen.c, secret.rs:118-178), bit for bit (all four
    components, including rejection-sampled rows), and a Detector built straight from the
    device-resident key gives the same detect output as the oracle."""
    a_sk, _, dk = PL.keys()
    ref = O.SecretPack.generate(PL.SK_SEED).generate_detection_key(PL.KEY_SEED, nthreads=16)
    parts = [(dk.bsk1, 4), (dk.ksk, 4), (dk.bsk2, 8), (dk.trace_key, 8)]
    bufs = [_dev_u(h.size, it) for h, it in parts]
    a_sk.generate_detection_key_device(PL.KEY_SEED, *[b.data_ptr() for b in bufs])
    for (h, _), b, r in zip(parts, bufs, ref):
        assert np.array_equal(_host(b, h.dtype).reshape(h.shape), r)
    mask = np.zeros(6, bool)
    mask[[1, 4]] = True
    ca, cb = PL.mixed_clues(mask, seed=77)
    orc = O.OracleDetector(*ref)
    want = orc.detect_batch(ca, cb, nthreads=6)
    orc.close()
    det = A.Detector.from_device_key(*[b.data_ptr() for b in bufs])
    del bufs  # the context holds its own converted copy
    assert np.array_equal(det.detect_batch(ca, cb), want)


def test_level1_rotations_both_paths(real, path):
    """omr_blind_rotate_level1 (full RLWE output) on explicit LWEs, incl. a = 0 steps and the
    extreme phases, bit-exact against the oracle's blind rotation."""
    _, det, orc = real
    rng = np.random.default_rng(17)
    la = rng.integers(0, 2048, (5, A.N0)).astype(np.uint16)
    la[1, ::3] = 0
    lb = np.array([0, 1, 1023, 1024, 2047], np.uint16)
    got = det.blind_rotate_level1(la, lb)
    for m in range(5):
        assert np.array_equal(got[m], orc.br1(la[m], lb[m])), f"rotation {m}"


def test_edge_inputs_bit_exact(real, path):
    """Inputs the KATs never produce, bit-exact against the oracle: all-zero clues (every CMUX
    step has a_i = 0), all-maximal clues (a_i = 2047), uniformly random clue words (not
    encryptions), and a ragged batch split into chunks of 5 (12 = 5 + 5 + 2, and 7 rotations per
    message so the level-1 workgroups of 4 rotations straddle messages). D = 0 is a no-op."""
    _, det, orc = real
    rng = np.random.default_rng(99)
    cases = [
        (np.zeros((2, A.N0), np.uint16), np.zeros((2, A.CLUE_COUNT), np.uint16)),
        (np.full((2, A.N0), 2047, np.uint16), np.full((2, A.CLUE_COUNT), 2047, np.uint16)),
        (rng.integers(0, 2048, (3, A.N0)).astype(np.uint16), rng.integers(0, 2048, (3, A.CLUE_COUNT)).astype(np.uint16)),
    ]
    for ca, cb in cases:
        assert np.array_equal(det.detect_batch(ca, cb), orc.detect_batch(ca, cb))
    mask = rng.random(12) < 0.5
    ca, cb = PL.mixed_clues(mask, seed=4321, first=1000)
    det.set_batch(5)
    try:
        got = det.detect_batch(ca, cb)
        # detect_with_time_info over host buffers staged in pieces of the batch size: the stage
        # times and the message count cover the whole call, not only its last piece
        got_t, info = det.detect_with_time_info(ca, cb)
    finally:
        det.set_batch(0)
    assert np.array_equal(got, orc.detect_batch(ca, cb))
    assert np.array_equal(got_t, got)
    assert info["messages"] == 12 and info["first_level_ms"] > info["key_switch_ms"] > 0
    assert info["second_level_ms"] > 0 and info["trace_ms"] > 0 and info["trace_separate"] == 1
    assert abs(info["total_ms"] - info["first_level_ms"] - info["second_level_ms"] - info["trace_ms"]) < 1e-3 * info["total_ms"] + 1e-3
    empty = det.detect_batch(np.zeros((0, A.N0), np.uint16), np.zeros((0, A.CLUE_COUNT), np.uint16))
    assert empty.shape == (0, 2, A.N2)
