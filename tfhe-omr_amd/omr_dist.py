"""Multi-GPU orchestration of the OMR detector: one process per GPU (torch.distributed; the
"nccl" backend is RCCL over xGMI on MI355X), messages sharded by contiguous global-index
ranges, no data-path collective for detect, and one reduce of the partial digests.

Reference behaviour (examples/omr.rs:154-293): detect every message (:219-223), then
encode_pertinent_indices for each index ciphertext (:239-242) and encode_pertinent_payloads
once (:256-262) over the WHOLE board. Encoding is linear in the pertinency vector, so each
rank encodes its own range with global indices and the partial digests are summed mod q2.
The bucket choices and payload weights are functions of (seed, global index), so the
result is independent of the number of ranks.

The compute backend is any object with `detect_batch(clue_a, clue_b)`,
`encode_pertinent_indices(rp, pv, seed, ct, global_offset)` and
`encode_pertinent_payloads(pv, payloads, weights, rp, global_offset)` — the GPU `Detector`
in production; tests also plug in the CPU oracle to exercise the orchestration under gloo.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

Q2 = 1125899906826241


def shard_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """Contiguous [first, first+count) of global message indices owned by `rank`."""
    base, rem = divmod(total, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


@dataclass
class Digest:
    indices: np.ndarray   # u64 [n_idx_ct][2][2048]
    payloads: np.ndarray  # u64 [n_pay_ct][2][2048]


def reduce_digest(local: np.ndarray, dist=None, device=None, dst: int = 0) -> np.ndarray | None:
    """Sum partial digests over ranks (int64; each < q2 < 2^50, <= 8192 ranks stay exact) and
    reduce mod q2 on `dst`. Returns the digest on dst, None elsewhere."""
    import torch

    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return local % np.uint64(Q2)
    t = torch.from_numpy(local.astype(np.int64))
    if device is not None:
        t = t.to(device)
    dist.reduce(t, dst=dst, op=dist.ReduceOp.SUM)
    if dist.get_rank() != dst:
        return None
    return (t.cpu().numpy().astype(np.uint64)) % np.uint64(Q2)


def run_omr_shard(backend, clue_a, clue_b, payloads, first: int, total: int, rp, index_seed: int,
                  weights: np.ndarray, dist=None, device=None):
    """Detect + encode this rank's shard and reduce the digest to rank 0.

    clue_a/clue_b/payloads hold this rank's messages (global indices first..first+len).
    `rp` is the board-wide RetrievalParams (all_payloads_count == total); `weights` the
    board-wide payload weights (omr_payload_weights). Returns (pv, Digest or None)."""
    pv = backend.detect_batch(clue_a, clue_b)
    idx = np.stack([backend.encode_pertinent_indices(rp, pv, index_seed, ct, first)
                    for ct in range(rp.max_encode_indices_cipher_count)])
    pay = backend.encode_pertinent_payloads(pv, payloads, weights, rp, first)
    local = np.concatenate([idx, pay]).astype(np.uint64)
    red = reduce_digest(local, dist, device)
    if red is None:
        return pv, None
    n = idx.shape[0]
    return pv, Digest(indices=red[:n], payloads=red[n:])
