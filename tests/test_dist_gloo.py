"""world_size-2 gloo test of the multi-GPU orchestration (tfhe-omr_amd/omr_dist.py) on CPU.
The compute backend is the CPU oracle (test-only); the shard plan, global offsets, encode +
digest reduce (omr_dist.encode_and_reduce, the function bench.py calls with the GPU backend)
are the production code. The 2-rank digest must equal the 1-rank digest bit-for-bit and decode
to the pertinent indices and payloads (omr_time_analyze.rs:215-235)."""
import os
import socket

import numpy as np
import pytest

import oracle_lib as O
import product_lib as PL
import retriever as R
from product_lib import omr_amd as A

import omr_dist

TOTAL = 6
MASK = np.array([0, 1, 0, 0, 1, 0], dtype=bool)
INDEX_SEED = 77
WSEED = bytes(range(5, 37))


class OracleBackend:
    """omr_dist backend interface on the CPU oracle (host numpy buffers, torch CPU digest)."""

    def __init__(self, dk):
        self.det = O.OracleDetector(dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key)

    def synchronize(self):
        pass

    def detect(self, ca, cb):
        return self.det.detect_batch(ca, cb, nthreads=2)

    def encode(self, pv, payloads, first, total, rp, seed, w):
        import torch
        idx = [O.encode_indices(pv, first, total, seed, ct) for ct in range(rp.max_encode_indices_cipher_count)]
        pay = O.encode_payloads(pv, payloads, first, total, w, rp.cmb_cipher_count, rp.cmb_count_per_cipher)
        return torch.from_numpy(np.concatenate([np.stack(idx), pay]).astype(np.int64))


def shard_inputs(first, count):
    a, b, _ = PL.keys()
    ca, cb = a.gen_clues(500, first, count)
    na, nb = b.gen_clues(501, first, count)
    m = MASK[first:first + count]
    ca[~m], cb[~m] = na[~m], nb[~m]
    pay = np.stack([np.random.default_rng(1000 + g).integers(0, 256, 612) for g in range(first, first + count)])
    return ca, cb, pay.astype(np.uint16)


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    _, _, dk = PL.keys()
    rp = A.RetrievalParams(TOTAL, int(MASK.sum()))
    w = A.payload_weights(WSEED, rp)
    first, count, total = omr_dist.plan(rank, world, total=TOTAL)
    assert total == TOTAL
    ca, cb, pay = shard_inputs(first, count)
    _, dg = omr_dist.run_omr_shard(OracleBackend(dk), ca, cb, pay, first, TOTAL, rp, INDEX_SEED, w, dist=dist)
    if rank == 0:
        np.savez(os.path.join(out_dir, f"digest_{world}.npz"), idx=dg.indices, pay=dg.payloads)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_plan_weak_and_strong():
    assert omr_dist.plan(3, 8, per_gpu=65536) == (3 * 65536, 65536, 524288)
    spans = [omr_dist.plan(r, 4, total=524288) for r in range(4)]
    assert spans == [(r * 131072, 131072, 524288) for r in range(4)]
    assert [omr_dist.plan(r, 3, total=10)[:2] for r in range(3)] == [(0, 4), (4, 3), (7, 3)]
    with pytest.raises(ValueError):
        omr_dist.plan(0, 1)
    with pytest.raises(ValueError):
        omr_dist.plan(0, 1, per_gpu=1, total=1)


def test_shard_range_partitions():
    for total in (1, 6, 65536, 2**20 + 3):
        for world in (1, 2, 3, 8):
            spans = [omr_dist.shard_range(r, world, total) for r in range(world)]
            assert spans[0][0] == 0 and sum(c for _, c in spans) == total
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def test_launch_envs_ranks_and_mismatch():
    """bench.py --gpus N: N rank environments when no launcher set WORLD_SIZE; none when a launcher
    did (and it agrees) or N == 1; an error when WORLD_SIZE disagrees with N."""
    base = {"PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    envs = omr_dist.launch_envs(4, base, 29600)
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["LOCAL_RANK"] == e["RANK"] and e["WORLD_SIZE"] == "4" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29600" for e in envs)
    assert all(e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/usr/bin" for e in envs)
    assert "RANK" not in base  # the caller's mapping is not modified
    assert omr_dist.launch_envs(1, base, 1) is None
    assert omr_dist.launch_envs(8, dict(base, WORLD_SIZE="8", RANK="3"), 1) is None
    assert omr_dist.launch_envs(1, dict(base, WORLD_SIZE="1"), 1) is None
    with pytest.raises(ValueError):
        omr_dist.launch_envs(8, dict(base, WORLD_SIZE="1"), 1)
    with pytest.raises(ValueError):
        omr_dist.launch_envs(2, dict(base, WORLD_SIZE="4"), 1)
    with pytest.raises(ValueError):
        omr_dist.launch_envs(0, base, 1)


def test_spawn_ranks_runs_every_rank_and_propagates_failure(tmp_path):
    import sys
    script = tmp_path / "child.py"
    script.write_text(
        "import os, sys, time\n"
        "r = os.environ['RANK']\n"
        "open(os.path.join(sys.argv[1], 'rank' + r), 'w').write(os.environ['WORLD_SIZE'] + ' ' + os.environ['LOCAL_RANK'])\n"
        "if len(sys.argv) > 2 and r == sys.argv[2]:\n"
        "    sys.exit(3)\n"
        "if len(sys.argv) > 2:\n"
        "    time.sleep(30)\n")
    envs = omr_dist.launch_envs(3, dict(os.environ, WORLD_SIZE=""), 29601)
    assert omr_dist.spawn_ranks([sys.executable, str(script), str(tmp_path)], envs, poll_s=0.05) == 0
    assert sorted(p.name for p in tmp_path.glob("rank*")) == ["rank0", "rank1", "rank2"]
    assert (tmp_path / "rank2").read_text() == "3 2"
    # rank 1 fails: the others (sleeping) are terminated and its code is returned promptly
    import time
    t = time.perf_counter()
    assert omr_dist.spawn_ranks([sys.executable, str(script), str(tmp_path), "1"], envs, poll_s=0.05) == 3
    assert time.perf_counter() - t < 20


def test_bench_rejects_gpus_world_size_mismatch():
    """bench.py exits non-zero (before touching a GPU) when WORLD_SIZE disagrees with --gpus."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8"],
                       env=dict(os.environ, WORLD_SIZE="1"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr and r.stdout == ""


@pytest.mark.slow
def test_two_rank_digest_equals_one_rank(tmp_path):
    import torch.multiprocessing as mp
    PL.keys()  # build keys once in the parent (workers rebuild deterministically)
    for world in (1, 2):
        mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    d1 = np.load(tmp_path / "digest_1.npz")
    d2 = np.load(tmp_path / "digest_2.npz")
    assert np.array_equal(d1["idx"], d2["idx"]) and np.array_equal(d1["pay"], d2["pay"])
    # the reduced digest decodes to the pertinent set and payloads
    a, _, _ = PL.keys()
    s2 = a.export()["s2"]
    rp = A.RetrievalParams(TOTAL, int(MASK.sum()))
    found = R.decode_indices(s2, d2["idx"], vars(rp), int(MASK.sum()))
    assert found == set(np.nonzero(MASK)[0].tolist())
    w = A.payload_weights(WSEED, rp)
    _, _, pay = shard_inputs(0, TOTAL)
    solved = R.decode_payloads(s2, d2["pay"], w, TOTAL, sorted(found), rp.combination_count)
    for i, p in zip(sorted(found), solved):
        assert p == pay[i].tolist()


def test_host_rendezvous_gloo_ranks(tmp_path):
    """bench.py's launcher path: the parent hosts the TCPStore on a port it keeps bound and the
    ranks (env:// rendezvous as agent-store clients) form a gloo group and all-reduce."""
    import sys
    script = tmp_path / "rank.py"
    script.write_text(
        "import os, sys, torch, torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "t = torch.tensor([float(dist.get_rank() + 1)])\n"
        "dist.all_reduce(t)\n"
        "open(os.path.join(sys.argv[1], 'sum' + os.environ['RANK']), 'w').write(str(int(t.item())))\n"
        "dist.destroy_process_group()\n")
    envs = omr_dist.launch_envs(3, dict(os.environ, WORLD_SIZE=""))
    store = omr_dist.host_rendezvous(envs)
    assert all(e["MASTER_PORT"] == str(store.port) and e["TORCHELASTIC_USE_AGENT_STORE"] == "True" for e in envs)
    assert omr_dist.spawn_ranks([sys.executable, str(script), str(tmp_path)], envs, poll_s=0.05) == 0
    del store
    assert [(tmp_path / f"sum{r}").read_text() for r in range(3)] == ["6", "6", "6"]


def test_bench_rank_failure_propagates():
    """bench.py --gpus 2 --one-device (the one-GPU rehearsal of the N > 1 path): a rank that dies
    after the rendezvous makes the launcher exit non-zero (here on CPU; the full path runs on the
    GPU in tests/test_gpu_sharded.py)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMR_BENCH_FAIL_RANK="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--one-device",
                        "--messages", "64"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "rank 1 failing on request" in r.stderr and r.stdout == "", r.stderr[-2000:]


def test_bench_hung_rank_times_out():
    """bench.py --gpus 2 --one-device with rank 1 never reaching the first collective
    (OMR_BENCH_HANG_RANK, a test hook): rank 0's barrier fails after --dist-timeout seconds, and the
    launcher exits non-zero and kills the hung rank, well inside the limit a driver would apply
    (a stuck rank must not hold an 8-GPU run until the driver's timeout)."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMR_BENCH_HANG_RANK="1")
    env.pop("WORLD_SIZE", None)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--one-device",
                        "--messages", "64", "--dist-timeout", "8"], env=env, capture_output=True, text=True,
                       timeout=240)
    took = time.monotonic() - t0
    assert r.returncode != 0 and r.stdout == "", r.stderr[-2000:]
    assert "rank 1 hanging on request" in r.stderr
    assert took < 120, took
