"""Multi-GPU orchestration of the OMR detector: one process per GPU (torch.distributed; the
"nccl" backend is RCCL over xGMI on MI355X), messages sharded by contiguous global-index
ranges, no data-path collective for detect, and one reduce of the partial digests.

Reference behaviour (examples/omr.rs): detect every message (`par_iter().map(detect)`,
:160-164), then encode_pertinent_indices for each index ciphertext and
encode_pertinent_payloads once over the WHOLE board (:180-203). Encoding is linear in the
pertinency vector, so each rank encodes its own range with global indices and the partial
digests are summed mod q2. The bucket choices and payload weights are functions of (seed,
global index), so the result is independent of the number of ranks.

bench.py and tests/test_dist_gloo.py both drive `run_omr_shard` / `encode_and_reduce`; the
compute backend is `GpuBackend` (libomr_gpu.so on device buffers) in production, and a CPU
oracle backend in the gloo test. A backend provides:
    detect(clue_a, clue_b) -> pertinency vector (backend-native buffer, D x 2 x 2048)
    encode(pv, payloads, first, total, rp, index_seed, weights) -> torch.int64 tensor
        [n_idx + n_pay][2][2048] of canonical partial digests (index ciphertexts first)
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np

Q2 = 1125899906826241


def launch_envs(gpus: int, environ, port: int = 0, addr: str = "127.0.0.1"):
    """Per-rank environments for a one-process-per-GPU run of `gpus` ranks, or None when this
    process is already a rank (WORLD_SIZE set, e.g. by torch.distributed.run) or gpus == 1.
    The reference sweeps worker counts inside one program (omr_time_analyze.rs:62-101); here
    `bench.py --gpus N` without an external launcher starts N ranks itself. Raises ValueError
    when WORLD_SIZE is set and disagrees with `gpus` (a SCALE record must not silently be a
    1-GPU number)."""
    if gpus < 1:
        raise ValueError(f"--gpus must be >= 1, got {gpus}")
    ws = environ.get("WORLD_SIZE")
    if ws is not None and ws != "":
        if int(ws) != gpus:
            raise ValueError(f"--gpus {gpus} but WORLD_SIZE={ws}: the launcher and the flag disagree")
        return None
    if gpus == 1:
        return None
    envs = []
    for r in range(gpus):
        e = dict(environ)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                 MASTER_ADDR=addr, MASTER_PORT=str(port))
        envs.append(e)
    return envs


def host_rendezvous(envs, addr: str = "127.0.0.1"):
    """Host the ranks' TCPStore in this launching process, on a port the OS picks and that stays
    bound for the whole run (a port probed and released before the ranks start could be taken by
    another process in between), and make every rank a client of it
    (TORCHELASTIC_USE_AGENT_STORE, the mechanism torch.distributed.run itself uses). Imports
    torch but touches no GPU. Returns the store: keep it alive until the ranks have exited."""
    from torch.distributed import TCPStore
    store = TCPStore(addr, 0, len(envs), True, wait_for_workers=False)
    for e in envs:
        e.update(MASTER_ADDR=addr, MASTER_PORT=str(store.port), TORCHELASTIC_USE_AGENT_STORE="True")
    return store


def spawn_ranks(argv, envs, poll_s: float = 0.02) -> int:
    """Start one child per environment running `argv` (stdout/stderr inherited: only rank 0
    prints the result line) and wait for all of them. If any child fails, the others are
    terminated and its exit code is returned; 0 when all succeed. The poll interval is short so
    that the first child to fail is the one reported: a peer whose collective then breaks exits
    (with its own code) a few hundred ms later, and with a 0.5 s interval both could land in one
    sweep, reported in rank order (profiles/r05zp/gpu_tests.log)."""
    import subprocess
    procs = [subprocess.Popen(argv, env=e) for e in envs]
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in procs:
                        q.terminate()
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    return rc


def shard_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """Contiguous [first, first+count) of global message indices owned by `rank`."""
    base, rem = divmod(total, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def plan(rank: int, world: int, per_gpu: int | None = None, total: int | None = None):
    """(first, count, total) of this rank. Weak scaling: `per_gpu` messages on every rank
    (total = per_gpu * world). Strong scaling: `total` messages split over the ranks."""
    if (per_gpu is None) == (total is None):
        raise ValueError("give exactly one of per_gpu (weak scaling) or total (strong scaling)")
    if per_gpu is not None:
        return rank * per_gpu, per_gpu, per_gpu * world
    first, count = shard_range(rank, world, total)
    return first, count, total


@dataclass
class Digest:
    indices: np.ndarray   # u64 [n_idx_ct][2][2048]
    payloads: np.ndarray  # u64 [n_pay_ct][2][2048]


def _on_backend(t, dist):
    """`t` where the process group's backend can reduce it: host memory for gloo."""
    if t.is_cuda and dist.get_backend() == "gloo":
        return t.cpu()
    return t


def reduce_digest(local, dist=None, dst: int = 0):
    """Sum the partial digests (torch.int64 [n_ct][2][2048], canonical < q2 < 2^50; the int64
    sum is exact up to 8,192 ranks) over the ranks with one reduce, and reduce mod q2 on `dst`.
    Returns the digest (numpy u64) on dst, None elsewhere. RCCL reduces `local` where it is
    (device memory); a gloo group gets device partials staged to host memory first (gloo has no
    device tensors), so the GPU backend also runs under gloo (tests/test_dist_gpu.py)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        local = _on_backend(local, dist)
        dist.reduce(local, dst=dst, op=dist.ReduceOp.SUM)
        if dist.get_rank() != dst:
            return None
    return local.cpu().numpy().view(np.uint64) % np.uint64(Q2)


def encode_and_reduce(backend, pv, payloads, first: int, total: int, rp, index_seed: int, weights,
                      dist=None, dst: int = 0):
    """encode_pertinent_indices (every index ciphertext) + encode_pertinent_payloads over this
    rank's shard with global indices, then the digest reduce. Returns (Digest or None on the
    other ranks, {"encode_s", "encode_reduce_s"} as the max over ranks)."""
    import torch

    if dist is not None and dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    local = backend.encode(pv, payloads, first, total, rp, index_seed, weights)
    backend.synchronize()
    t1 = time.perf_counter()
    red = reduce_digest(local, dist, dst)
    backend.synchronize()
    t2 = time.perf_counter()
    times = [t1 - t0, t2 - t0]
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        tt = _on_backend(torch.tensor(times, dtype=torch.float64, device=local.device), dist)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        times = tt.tolist()
    timing = {"encode_s": times[0], "encode_reduce_s": times[1]}
    if red is None:
        return None, timing
    n = rp.max_encode_indices_cipher_count
    return Digest(indices=red[:n], payloads=red[n:]), timing


def run_omr_shard(backend, clue_a, clue_b, payloads, first: int, total: int, rp, index_seed: int,
                  weights, dist=None):
    """Detect + encode this rank's shard (global indices first..first+len) and reduce the digest
    to rank 0. `rp` is the board-wide RetrievalParams (all_payloads_count == total); `weights`
    the board-wide payload weights (omr_payload_weights). Returns (pv, Digest or None)."""
    pv = backend.detect(clue_a, clue_b)
    digest, _ = encode_and_reduce(backend, pv, payloads, first, total, rp, index_seed, weights, dist)
    return pv, digest


class GpuBackend:
    """libomr_gpu.so on device buffers (torch tensors on `device`), enqueued on `stream`."""

    def __init__(self, detector, device, stream):
        self.det = detector
        self.device = device
        self.stream = stream
        self._weights = None

    def synchronize(self):
        """Wait for the stream and surface any device-side failure of the detect calls."""
        self.det.check(self.stream.cuda_stream)

    def detect(self, clue_a, clue_b, out=None):
        """clue_a int16 [D][512], clue_b int16 [D][7] device tensors -> pv int64 [D][2][2048]."""
        import torch
        D = clue_a.shape[0]
        if out is None:
            out = torch.empty((D, 2, 2048), dtype=torch.int64, device=self.device)
        self.det.detect_batch_device(clue_a.data_ptr(), clue_b.data_ptr(), D, out.data_ptr(),
                                     self.stream.cuda_stream)
        return out

    def encode(self, pv, payloads, first, total, rp, index_seed, weights):
        import torch
        n_idx, n_pay, per = rp.max_encode_indices_cipher_count, rp.cmb_cipher_count, rp.cmb_count_per_cipher
        D = pv.shape[0]
        if self._weights is None or self._weights[0] is not weights:
            self._weights = (weights, torch.from_numpy(np.ascontiguousarray(weights).view(np.int16)).to(self.device))
        d_w = self._weights[1]
        d_pay = payloads if isinstance(payloads, torch.Tensor) else \
            torch.from_numpy(np.ascontiguousarray(payloads, dtype=np.uint16).view(np.int16)).to(self.device)
        dig = torch.empty((n_idx + n_pay, 2, 2048), dtype=torch.int64, device=self.device)
        s = self.stream.cuda_stream
        self.det.encode_indices_device(pv.data_ptr(), D, first, total, index_seed, 0, n_idx, dig.data_ptr(), s)
        self.det.encode_payloads_device(pv.data_ptr(), d_pay.data_ptr(), D, first, total, d_w.data_ptr(), n_pay,
                                        per, dig[n_idx:].data_ptr(), s)
        return dig
