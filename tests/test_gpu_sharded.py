"""GPU tests of the sharded / multi-context paths on one MI355X.

- Two ranks on one GPU: two gloo processes, both on cuda:0, run omr_dist.run_omr_shard with the
  production GpuBackend over contiguous global-index shards (D = 2 x 4,096); the reduced digest
  must equal the 1-rank digest, the oracle's encode_pertinent_indices / _payloads on the full
  pertinency vector, and decode to the pertinent set and payloads (examples/omr.rs:160-203,
  omr_time_analyze.rs:215-235).
- configs[4]'s digest at D = 2^20: 8 sequential shards of 131,072 messages on one context through
  omr_dist.encode_and_reduce(dist=None), partial digests summed mod q2, 50/50 indices and payloads
  recovered; shard-boundary messages bit-exact against the oracle.
- Two contexts, two streams, concurrent 64-message latency chunks (two-CU cooperative kernel),
  bit-exact against the throughput kernels; omr_ctx_check reports no error.
- DetectTimeInfo split (detector.rs:169-221): timing mode 2 gives the trace its own time on the
  throughput path, with an identical output.
"""
import os
import socket

import torch  # noqa: F401  (before libomr_gpu.so: one HIP runtime per process, conftest.py)
import numpy as np
import pytest

import oracle_lib as O
import product_lib as PL
import retriever as R
from product_lib import omr_amd as A

import omr_dist

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)
INDEX_SEED = 9
WEIGHT_SEED = bytes(range(1, 33))


def synthetic_payloads(first: int, count: int) -> np.ndarray:
    """bench.py's payloads: a fixed function of the global message index, u16 [count][612] < 256."""
    i = np.arange(first, first + count, dtype=np.uint64)[:, None]
    b = np.arange(612, dtype=np.uint64)[None, :]
    h = i * np.uint64(0x9E3779B97F4A7C15) + b * np.uint64(0xBF58476D1CE4E5B9)
    h ^= h >> np.uint64(31)
    return ((h >> np.uint64(24)) & np.uint64(255)).astype(np.uint16)


def device_detector(dev):
    """bench.py's seeded device keys (pack 42, key seed 7) and a Detector over them."""
    pack_a, pack_b = A.SecretKeyPack(PL.SK_SEED), A.SecretKeyPack(PL.SK2_SEED)
    cur = torch.cuda.current_stream(dev).cuda_stream
    kb = [torch.empty(int(np.prod(s)), dtype=dt, device=dev)
          for s, dt in ((A.BSK1_SHAPE, torch.int32), (A.KSK_SHAPE, torch.int32),
                        (A.BSK2_SHAPE, torch.int64), (A.TK_SHAPE, torch.int64))]
    pack_a.generate_detection_key_device(PL.KEY_SEED, *[b.data_ptr() for b in kb], stream=cur)
    det = A.Detector.from_device_key(*[b.data_ptr() for b in kb], device=dev.index or 0)
    del kb  # the context keeps its converted copy
    return pack_a, pack_b, det


def device_clues(pack_a, pack_b, first, count, mask, dev):
    """Clues of global indices [first, first + count): pack A (seed 1000) where pertinent, else B."""
    ca = torch.empty((count, A.N0), dtype=torch.int16, device=dev)
    cb = torch.empty((count, A.CLUE_COUNT), dtype=torch.int16, device=dev)
    na, nb = torch.empty_like(ca), torch.empty_like(cb)
    cur = torch.cuda.current_stream(dev).cuda_stream
    pack_a.gen_clues_device(1000, first, count, ca.data_ptr(), cb.data_ptr(), stream=cur)
    pack_b.gen_clues_device(1001, first, count, na.data_ptr(), nb.data_ptr(), stream=cur)
    m = torch.from_numpy(mask).to(dev)[:, None]
    return torch.where(m, ca, na).contiguous(), torch.where(m, cb, nb).contiguous()


# ---- two ranks (gloo) on one GPU --------------------------------------------------------------
TWO_RANK_TOTAL = 2 * 4096


def two_rank_board():
    rng = np.random.default_rng(77)
    pert = np.sort(rng.choice(TWO_RANK_TOTAL, 50, replace=False))
    mask = np.zeros(TWO_RANK_TOTAL, dtype=bool)
    mask[pert] = True
    return pert, mask


def run_shard(dist, world, rank, dev, pack_a, pack_b, det, keep_pv=False):
    """omr_dist.run_omr_shard on this rank's contiguous shard with the production GpuBackend."""
    pert, mask = two_rank_board()
    first, count, total = omr_dist.plan(rank, world, total=TWO_RANK_TOTAL)
    rp = A.RetrievalParams(total, len(pert))
    w = A.payload_weights(WEIGHT_SEED, rp)
    det.set_latency_threshold(0)
    d_ca, d_cb = device_clues(pack_a, pack_b, first, count, mask[first:first + count], dev)
    backend = omr_dist.GpuBackend(det, dev, torch.cuda.current_stream(dev))
    pv, dg = omr_dist.run_omr_shard(backend, d_ca, d_cb, synthetic_payloads(first, count), first, total, rp,
                                    INDEX_SEED, w, dist=dist)
    return (pv.cpu().numpy().view(np.uint64) if keep_pv else None), dg


def _two_rank_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pack_a, pack_b, det = device_detector(dev)
    _, dg = run_shard(dist, world, rank, dev, pack_a, pack_b, det)
    if rank == 0:
        np.savez(os.path.join(out_dir, f"digest_{world}.npz"), idx=dg.indices, pay=dg.payloads)
    dist.barrier()
    det.close()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_one_gpu_gloo_digest(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_two_rank_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    d2 = np.load(tmp_path / "digest_2.npz")
    dev = torch.device("cuda", 0)
    pack_a, pack_b, det = device_detector(dev)
    pv, d1 = run_shard(None, 1, 0, dev, pack_a, pack_b, det, keep_pv=True)
    det.close()
    assert np.array_equal(d1.indices, d2["idx"]) and np.array_equal(d1.payloads, d2["pay"])
    pert, mask = two_rank_board()
    rp = A.RetrievalParams(TWO_RANK_TOTAL, len(pert))
    for ct in range(rp.max_encode_indices_cipher_count):
        assert np.array_equal(d2["idx"][ct], O.encode_indices(pv, 0, TWO_RANK_TOTAL, INDEX_SEED, ct)), f"index ct {ct}"
    w = A.payload_weights(WEIGHT_SEED, rp)
    pay = synthetic_payloads(0, TWO_RANK_TOTAL)
    last = rp.cmb_cipher_count - 1
    assert np.array_equal(d2["pay"][:1], O.encode_payloads(pv, pay, 0, TWO_RANK_TOTAL, w, 1, 2))
    wl = w[2 * last * TWO_RANK_TOTAL:]
    assert np.array_equal(d2["pay"][last:], O.encode_payloads(pv, pay, 0, TWO_RANK_TOTAL, wl, 1, 2))
    indices, pays = A.Retriever(rp, pack_a).decode_digest(d2["idx"], d2["pay"], WEIGHT_SEED)
    assert indices == pert.tolist()
    assert np.array_equal(pays, pay[pert])


# ---- configs[4]: D = 2^20 as 8 shards of 131,072 on one context --------------------------------
C4_TOTAL, C4_SHARDS = 1 << 20, 8
C4_PER = C4_TOTAL // C4_SHARDS


class Config4:
    """configs[4]'s board on one context. shard(k) detects and encodes shard k once (memoised) and
    returns its partial digest plus the boundary / pertinent messages it checked, so every test
    below is self-contained: any -k selection runs the shards it needs."""

    def __init__(self):
        self.dev = torch.device("cuda", 0)
        torch.cuda.set_device(self.dev)
        self.pack_a, self.pack_b, self.det = device_detector(self.dev)
        self.det.set_batch(65536)  # bench.py's launch size
        rng = np.random.default_rng(2025)  # bench.py's pertinent set for D = 2^20
        self.pert = np.sort(rng.choice(C4_TOTAL, 50, replace=False))
        self.mask = np.zeros(C4_TOTAL, dtype=bool)
        self.mask[self.pert] = True
        self.rp = A.RetrievalParams(C4_TOTAL, len(self.pert))
        assert (self.rp.max_encode_indices_cipher_count, self.rp.cmb_cipher_count) == (8, 28)
        self.w = A.payload_weights(WEIGHT_SEED, self.rp)
        self.backend = omr_dist.GpuBackend(self.det, self.dev, torch.cuda.current_stream(self.dev))
        self.pv = torch.empty((C4_PER, 2, 2048), dtype=torch.int64, device=self.dev)
        self.parts = {}

    def shard(self, k):
        if k in self.parts:
            return self.parts[k]
        first = k * C4_PER
        mask = self.mask[first:first + C4_PER]
        d_ca, d_cb = device_clues(self.pack_a, self.pack_b, first, C4_PER, mask, self.dev)
        self.backend.detect(d_ca, d_cb, out=self.pv)
        self.backend.synchronize()
        # shard-boundary messages (global first, first + 131,071) and a pertinent one
        local = sorted({0, C4_PER - 1} | ({int(np.nonzero(mask)[0][0])} if mask.any() else set()))
        idx = torch.tensor(local, device=self.dev)
        checked = (d_ca[idx].cpu().numpy().view(np.uint16), d_cb[idx].cpu().numpy().view(np.uint16),
                   self.pv[idx].cpu().numpy().view(np.uint64), [first + m for m in local])
        dg, _ = omr_dist.encode_and_reduce(self.backend, self.pv, synthetic_payloads(first, C4_PER), first, C4_TOTAL,
                                           self.rp, INDEX_SEED, self.w, dist=None)
        self.parts[k] = (np.concatenate([dg.indices, dg.payloads]), checked)
        return self.parts[k]


@pytest.fixture(scope="module")
def c4():
    board = Config4()
    yield board
    board.det.close()


@pytest.mark.parametrize("shard", range(C4_SHARDS))
def test_config4_shard(c4, shard):
    """Shard `shard` of configs[4]: its boundary messages and one pertinent message bit-exact vs the oracle."""
    _, (ca, cb, got, gidx) = c4.shard(shard)
    _, _, dk = PL.keys()
    orc = O.OracleDetector(dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key)
    want = orc.detect_batch(ca, cb, nthreads=THREADS)
    orc.close()
    for k, g in enumerate(gidx):
        assert np.array_equal(got[k], want[k]), f"global message {g} differs from the oracle"


@pytest.mark.timeout(900)  # alone (e.g. -k digest_sum) it runs all eight 131,072-message shards
def test_config4_digest_sum_recovers_board(c4):
    """The mod-q2 sum of the eight shards' partial digests (what the 8-GPU run reduces with RCCL)
    recovers all 50 pertinent indices and their payloads."""
    digest = None
    for k in range(C4_SHARDS):
        part, _ = c4.shard(k)
        digest = part.copy() if digest is None else (digest + part) % np.uint64(A.Q2)
    rp, n = c4.rp, c4.rp.max_encode_indices_cipher_count
    indices, pays = A.Retriever(rp, c4.pack_a).decode_digest(digest[:n], digest[n:], WEIGHT_SEED)
    assert indices == c4.pert.tolist()
    want = np.concatenate([synthetic_payloads(int(i), 1) for i in indices])
    assert np.array_equal(pays, want)


# ---- concurrent contexts, latency path ---------------------------------------------------------
def test_two_contexts_concurrent_latency_chunks():
    """Two contexts on two streams each run a 64-message chunk on the latency kernels at the same
    time (two cooperative two-CU grids of 128 workgroups); both outputs equal the throughput
    kernels' bit for bit and omr_ctx_check reports no hand-off error."""
    a, b, dk = PL.keys()
    s2 = a.export()["s2"]
    dets = [A.Detector(dk), A.Detector(dk)]
    n = 64
    masks = [np.arange(n) % 7 == k for k in (0, 3)]
    clues = [PL.mixed_clues(m, seed=7100 + 10 * k, first=1000 * k) for k, m in enumerate(masks)]
    d_in = [(torch.from_numpy(ca.view(np.int16)).cuda(), torch.from_numpy(cb.view(np.int16)).cuda()) for ca, cb in clues]
    outs = [torch.empty((n, 2, 2048), dtype=torch.int64, device="cuda:0") for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    for rep in range(3):
        for det, (dca, dcb), out, s in zip(dets, d_in, outs, streams):
            det.detect_batch_device(dca.data_ptr(), dcb.data_ptr(), n, out.data_ptr(), s.cuda_stream)
        for det, s in zip(dets, streams):
            det.check(s.cuda_stream)
        for k, det in enumerate(dets):
            det.set_latency_threshold(0)
            want = det.detect_batch(*clues[k])
            det.set_latency_threshold(64)
            got = outs[k].cpu().numpy().view(np.uint64)
            assert np.array_equal(got, want), f"context {k}, repetition {rep}"
            for m in range(n):
                dec = R.decrypt_decode(s2, got[m])
                assert (dec[0] == 1) == masks[k][m] and not dec[1:].any()
    for det in dets:
        det.close()


def test_detect_time_info_split():
    """Timing mode 2 (the reference's DetectTimeInfo split) runs the throughput path's level-2
    rotation and trace as two launches: identical output, the trace timed on its own, and the
    stages sum to the total; mode 1 likewise (since round 5 the production path runs the FFT trace
    as its own launch, trace_fft_kernel)."""
    a, b, dk = PL.keys()
    det = A.Detector(dk)
    det.set_latency_threshold(0)
    mask = np.arange(200) % 11 == 0
    ca, cb = PL.mixed_clues(mask, seed=8080)
    out2, t2 = det.detect_with_time_info(ca, cb)
    det.enable_timing(1)
    out1 = det.detect_batch(ca, cb)
    t1 = det.last_timing()
    det.enable_timing(0)
    plain = det.detect_batch(ca, cb)
    det.close()
    assert np.array_equal(out2, plain) and np.array_equal(out1, plain)
    assert t2["trace_separate"] == 1 and t2["trace_ms"] > 0 and t2["messages"] == 200
    assert t2["first_level_ms"] > t2["key_switch_ms"] > 0 and t2["second_level_ms"] > 0
    assert abs(t2["total_ms"] - t2["first_level_ms"] - t2["second_level_ms"] - t2["trace_ms"]) < 1e-3 * t2["total_ms"] + 1e-3
    assert t1["trace_separate"] == 1 and 0 < t1["trace_ms"] < 0.2 * t1["second_level_ms"]
    assert abs(t1["total_ms"] - t1["first_level_ms"] - t1["second_level_ms"] - t1["trace_ms"]) < 1e-3 * t1["total_ms"] + 1e-3


def _run_bench(args, env_extra=None, timeout=420):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, **(env_extra or {}))
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, "-u", os.path.join(root, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_two_ranks_one_device_rehearsal():
    """bench.py's own N > 1 path before the driver's 8-GPU run: --gpus 2
    through the real spawn path (the launcher hosts the rendezvous store), both ranks on cuda:0
    under a gloo group (--one-device; RCCL cannot run two ranks on one GPU): the barrier + MAX
    all-reduce timing, the digest reduce, rank 0's single JSON line, rank 1's early return."""
    import json
    r = _run_bench(["--gpus", "2", "--one-device", "--messages", "2048", "--steps", "1", "--warmup", "0",
                    "--batch", "2048"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    print("\n" + lines[0][:600])
    assert line["n_gpus"] == 2 and line["config"]["messages_total"] == 4096
    assert line["config"]["messages_per_gpu"] == 2048 and line["config"]["parallelism"] == "dp2"
    assert line["e2e"]["ok"] and line["e2e"]["pertinent_recovered"] == 50
    assert line["correct"] and line["exactness"]["certified"] and line["exactness"]["guarded_output_identical"]
    assert "cpu_baseline" not in line  # rank 0 of a 2-rank job reports no CPU leg
    assert all(not k.endswith("_frac") or v is None or v <= 1 for k, v in line["hbm"].items())
    # round 6: the group's own world size, every rank's timed region, the
    # per-step spread of both rotations, the fixed-work fractions
    assert line["dist"]["world_size_observed"] == 2 and line["dist"]["backend"] == "gloo"
    re_ = line["dist"]["rank_elapsed_s"]
    assert 0 < re_["min"] <= re_["max"] and abs(line["ms_per_step"] - re_["max"] * 1e3) < 1.0
    sp = line["per_step_spread"]
    assert sp["level1_rotation_ms"]["min"] > 0 and sp["level2_rotation_ms"]["max_over_min"] >= 1.0
    assert 0 < line["roofline"]["frac_fixed_work"] <= 1 and 0 < line["detect_fp64"]["detect_fp64_frac_fixed_work"] <= 1
    assert line["exactness"]["guarded_ms_per_step"] > 0


def test_bench_two_ranks_one_device_child_failure():
    """A rank that dies makes bench.py --gpus 2 exit non-zero with no result line."""
    r = _run_bench(["--gpus", "2", "--one-device", "--messages", "256", "--steps", "1", "--warmup", "0"],
                   env_extra={"OMR_BENCH_FAIL_RANK": "1"}, timeout=300)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == ""
