"""GPU parity at the geometry bench.py times, through the device entry points.

configs[2] (D = 65,536 in one 65,536-message launch, bench.py's default, and in the library's
default 16,384-message launches) and configs[4]'s per-GPU share (D = 131,072 in two launches)
run through omr_detect_batch_device on bench.py's seeded keys and clue streams (pack 42 /
pack 4242, clue seeds 1000 / 1001): every output must pass the omd.rs:48-58 KAT (pertinent ->
[1, 0, ..., 0], other -> 0) with the library retriever, and the messages at the launch
boundaries plus two pertinent ones must equal the CPU oracle bit for bit. Further cases cover
what the bench path relies on and the small-batch tests never reach: several device calls on
different streams sharing one context's scratch (and the host entry point between them), and
the encode kernels at D >= 16,384 with several ciphertexts, a global offset and a non-default
stream, against the oracle."""
import os

import numpy as np
import pytest

import oracle_lib as O
import product_lib as PL
from product_lib import omr_amd as A

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def ctx():
    a, b, dk = PL.keys()
    det = A.Detector(dk)
    orc = O.OracleDetector(dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key)
    yield a, b, det, orc
    det.close()
    orc.close()


def _device_clues(a, b, D, first, mask):
    """bench.py's clue streams on the device: pack A (seed 1000) where pertinent, else pack B (1001)."""
    import torch
    dev = torch.device("cuda", 0)
    ca = torch.empty((D, A.N0), dtype=torch.int16, device=dev)
    cb = torch.empty((D, A.CLUE_COUNT), dtype=torch.int16, device=dev)
    na, nb = torch.empty_like(ca), torch.empty_like(cb)
    a.gen_clues_device(1000, first, D, ca.data_ptr(), cb.data_ptr())
    b.gen_clues_device(1001, first, D, na.data_ptr(), nb.data_ptr())
    m = torch.from_numpy(mask).to(dev)[:, None]
    return torch.where(m, ca, na).contiguous(), torch.where(m, cb, nb).contiguous()


def _kat_all(a, d_out, mask, piece=8192):
    """omd.rs:48-58 on every output: decrypt + decode (library retriever, host chunks)."""
    ret = A.Retriever(A.RetrievalParams(len(mask), 1), a)
    for s in range(0, len(mask), piece):
        dec = ret.decrypt_decode(d_out[s:s + piece].cpu().numpy().view(np.uint64))
        assert np.array_equal(dec[:, 0] == 1, mask[s:s + piece]), f"pertinency bit wrong in [{s}, {s + piece})"
        assert not dec[:, 1:].any() and not dec[~mask[s:s + piece], 0].any(), f"nonzero slot in [{s}, {s + piece})"


@pytest.mark.parametrize("D,batch", [(65536, 65536), (65536, 16384), (131072, 65536)])
def test_timed_geometry_device_path(ctx, D, batch):
    import torch
    a, b, det, orc = ctx
    rng = np.random.default_rng(2025)
    pert = np.sort(rng.choice(D, 50, replace=False))
    mask = np.zeros(D, dtype=bool)
    mask[pert] = True
    d_ca, d_cb = _device_clues(a, b, D, 0, mask)
    d_out = torch.empty((D, 2, 2048), dtype=torch.int64, device="cuda:0")
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    det.set_batch(batch)  # bench.py's launch size (65,536) or the library default (16,384)
    with torch.cuda.stream(side):
        det.detect_batch_device(d_ca.data_ptr(), d_cb.data_ptr(), D, d_out.data_ptr(), side.cuda_stream)
    side.synchronize()
    det.set_batch(0)
    _kat_all(a, d_out, mask)
    picks = sorted({0, 16383, 16384, 32767, 49152, 65535, D - 1, int(pert[0]), int(pert[-1])} |
                   ({65536, 98304} if D > 65536 else set()))
    idx = torch.tensor(picks, device="cuda:0")
    ca = d_ca[idx].cpu().numpy().view(np.uint16)
    cb = d_cb[idx].cpu().numpy().view(np.uint16)
    got = d_out[idx].cpu().numpy().view(np.uint64)
    want = orc.detect_batch(ca, cb, nthreads=THREADS)
    for k, m in enumerate(picks):
        assert np.array_equal(got[k], want[k]), f"message {m} differs from the oracle"


def test_device_calls_on_two_streams_and_host_call(ctx):
    """Three detect calls enqueued back to back on one context without waiting: device buffers on
    stream s1, device buffers on stream s2, then the host entry point (context stream). Each is
    split into chunks of 10 (the multi-chunk offset loop of detect_device). The context's scratch
    is shared, so the later calls must wait for the earlier ones (omr_ctx::scratch_free)."""
    import torch
    a, b, det, orc = ctx
    D = 24
    masks = [np.arange(D) % 5 == k for k in range(3)]
    clues = [PL.mixed_clues(m, seed=3000 + 10 * k, first=100 * k) for k, m in enumerate(masks)]
    dev_in = [(torch.from_numpy(ca.view(np.int16)).cuda(), torch.from_numpy(cb.view(np.int16)).cuda())
              for ca, cb in clues[:2]]
    outs = [torch.empty((D, 2, 2048), dtype=torch.int64, device="cuda:0") for _ in range(2)]
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    det.set_batch(10)
    try:
        for (dca, dcb), out, s in zip(dev_in, outs, (s1, s2)):
            det.detect_batch_device(dca.data_ptr(), dcb.data_ptr(), D, out.data_ptr(), s.cuda_stream)
        host = det.detect_batch(*clues[2])
        torch.cuda.synchronize()
    finally:
        det.set_batch(0)
    got = [o.cpu().numpy().view(np.uint64) for o in outs] + [host]
    for k, (ca, cb) in enumerate(clues):
        assert np.array_equal(got[k], orc.detect_batch(ca, cb, nthreads=THREADS)), f"call {k}"


@pytest.mark.parametrize("max_chunks", [0, 7])
def test_encode_device_large_multi_ct(ctx, max_chunks):
    """encode_*_device at D = 20,000 (the 128-message-per-workgroup path), 5 index ciphertexts
    and 3 payload ciphertexts of 2 combinations, global offset 12,345 of a 100,000 board, on a
    side stream; bit-exact against the oracle and against the host entry points. max_chunks = 7
    gives 2,858 messages per workgroup, the regime of D > 524,288 at the default 4,096 chunks
    (the index kernel stages its bucket choices 128 messages at a time)."""
    import torch
    _, _, det, _ = ctx
    det.set_encode_chunks(max_chunks)
    D, off, allc = 20000, 12345, 100000
    rng = np.random.default_rng(5)
    pv = rng.integers(0, A.Q2, (D, 2, 2048), dtype=np.uint64)
    pay = rng.integers(0, 256, (D, 612)).astype(np.uint16)
    rp = A.RetrievalParams(allc, 50)
    n_idx, n_pay, per = 5, 3, 2
    rp.cmb_cipher_count, rp.cmb_count_per_cipher = n_pay, per
    w, _ = O.payload_weights(bytes(range(7, 39)), n_pay * per * allc)
    d_pv = torch.from_numpy(pv.view(np.int64)).cuda()
    d_pay = torch.from_numpy(pay.view(np.int16)).cuda()
    d_w = torch.from_numpy(w.view(np.int16)).cuda()
    d_idx = torch.empty((n_idx, 2, 2048), dtype=torch.int64, device="cuda:0")
    d_dig = torch.empty((n_pay, 2, 2048), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    det.encode_indices_device(d_pv.data_ptr(), D, off, allc, 9, 0, n_idx, d_idx.data_ptr(), s.cuda_stream)
    det.encode_payloads_device(d_pv.data_ptr(), d_pay.data_ptr(), D, off, allc, d_w.data_ptr(), n_pay, per,
                               d_dig.data_ptr(), s.cuda_stream)
    s.synchronize()
    idx = d_idx.cpu().numpy().view(np.uint64)
    dig = d_dig.cpu().numpy().view(np.uint64)
    for ct in (0, 4):
        assert np.array_equal(idx[ct], O.encode_indices(pv, off, allc, 9, ct)), f"index ct {ct}"
    assert np.array_equal(idx[2], det.encode_pertinent_indices(rp, pv, 9, 2, global_offset=off))
    assert np.array_equal(dig, O.encode_payloads(pv, pay, off, allc, w, n_pay, per))
    assert np.array_equal(dig, det.encode_pertinent_payloads(pv, pay, w, rp, global_offset=off))
    det.set_encode_chunks(0)


def test_encode_rejects_bad_shapes(ctx):
    _, _, det, _ = ctx
    pv = np.zeros((4, 2, 2048), np.uint64)
    rp = A.RetrievalParams(3, 1)  # board smaller than offset + D
    with pytest.raises(A.OmrError):
        det.encode_pertinent_indices(rp, pv, 9, 0)
