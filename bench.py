"""bench.py — detect-phase messages/s of the MI355X InstantOMR detector.

Workload (BASELINE.json configs[2]): full Detector::detect() (detector.rs:135-166) over
D = 65,536 synthetic clues per GPU (50 pertinent, the rest from a second sender key),
inputs resident in HBM, outputs (the pertinency vector, D x 32 KiB) written to HBM.
One step = one detect pass over the D clues of every rank. N > 1: one process per GPU
(torch.distributed, RCCL), each rank owns a contiguous range of global message indices
(weak scaling, no data-path collective). Rank 0 prints one JSON line.

After the timed detect steps, one end-to-end pass (configs[4] shape) runs
on the last pertinency vector: encode_pertinent_indices + encode_pertinent_payloads over each
rank's shard with global indices, one RCCL reduce of the partial digests to rank 0, and the
client-side retrieval (the library's Retriever) must recover exactly the pertinent indices and
their payloads ("e2e" in the JSON line; --no-e2e skips it).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--messages D] [--no-e2e]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tfhe-omr_amd"))

import omr_amd as A  # noqa: E402

# Algorithmic bytes per message (SURVEY.md §8d key-streaming model, reference u32/u64 formats):
# every evaluation-key element counted once per use by one message.
BR1_BYTES = 7 * 512 * 8 * 2 * 1024 * 4          # 7 x BSK1 (u32)            = 234,881,024
KS_BYTES = 1024 * 27 * 671 * 4                    # KSK (u32)                =  74,207,232
BR2_BYTES = 670 * 12 * 2 * 2048 * 8               # BSK2 (u64)               = 263,454,720
TRACE_BYTES = 11 * 25 * 2 * 2048 * 8              # trace key (u64)          =   9,011,200
IO_BYTES = 512 * 2 + 7 * 2 + 2 * 2048 * 8         # clue in + NttRlwe out    =      33,806
DETECT_BYTES = BR1_BYTES + KS_BYTES + BR2_BYTES + TRACE_BYTES + IO_BYTES
KERNEL_BYTES = {  # per message, per pipeline stage (kernel names from A.detect_kernels())
    "br1": BR1_BYTES + 7 * (512 * 2 + 2) + 7 * 1025 * 4,
    "ks": KS_BYTES + 1025 * 4 + 671 * 4,
    "br2": BR2_BYTES + TRACE_BYTES + 671 * 4 + 2 * 2048 * 8,
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
# FP64 VALU issue rate: 256 CUs x 4 SIMDs x 16 FP64 lanes x 2.4 GHz (78.6 TFLOP/s counting FMA as
# 2); the arithmetic microbenchmark reaches 95 % of it (profiles/r01_microbench_arith.txt).
FP64_PEAK_T_LANE_INSTR = 256 * 4 * 16 * 2.4e9 / 1e12
PUBLISHED_CPU_MSG_S = 1e3 / 234.073003  # README.md:122, 1 thread AVX-512


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--messages", type=int, default=65536, help="clues per GPU")
    ap.add_argument("--pertinent", type=int, default=50)
    ap.add_argument("--cpu-baseline-msgs", type=int, default=256)
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the RCCL process group even at world size 1 (rehearses the N > 1 path)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the encode + reduce + retrieval pass")
    return ap.parse_args()


def cpu_baseline(dk, ca, cb, nmsg):
    """The oracle detect() (oracle/, plain-C restatement of the reference path: kind "port")
    timed on this host's cores over a bounded sample (the Rust reference cannot be built
    here). Test infrastructure, used only for this reported leg."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    cores = min(16, os.cpu_count() or 1)
    det = O.OracleDetector(dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key)
    det.detect_batch(ca[:1], cb[:1], nthreads=1)  # warm the tables
    t = time.perf_counter()
    det.detect_batch(ca[:nmsg], cb[:nmsg], nthreads=cores)
    dt = time.perf_counter() - t
    det.close()
    return {"value": round(nmsg / dt, 3), "unit": "messages/s", "cores": cores, "kind": "port",
            "sample": f"{nmsg} detect() calls of the same workload, OpenMP over messages, {dt:.1f}s wall"}


def workload_name(D, world):
    """BASELINE.json config the run corresponds to (configs[2] at D = 65,536 per GPU, configs[3]
    at N = 8, configs[4]'s detect + encode shape at D = 2^20 over the job)."""
    name = f"full detect() D={D} per GPU, {D * world} total"
    if D == 65536:
        name += " (configs[2]; configs[3] at N=8)"
    elif D * world == 1 << 20:
        name += " (configs[4]: detect + encode + retrieval at D=2^20)"
    return name


def load_profile(name):
    """A committed rocprofv3 summary under profiles/ (tools/profile.sh, tools/compute_summary.py)."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def synthetic_payloads(first: int, count: int) -> np.ndarray:
    """Payloads (payload.rs:26-38: 612 bytes) as a fixed function of the global message index,
    so any rank (and the retrieval check) can regenerate them: u16 [count][612] in [0, 256)."""
    i = np.arange(first, first + count, dtype=np.uint64)[:, None]
    b = np.arange(612, dtype=np.uint64)[None, :]
    h = i * np.uint64(0x9E3779B97F4A7C15) + b * np.uint64(0xBF58476D1CE4E5B9)
    h ^= h >> np.uint64(31)
    return ((h >> np.uint64(24)) & np.uint64(255)).astype(np.uint16)


def end_to_end(det, pack_a, d_out, D, first, total, pert, dist, dev, stream, rank):
    """encode_pertinent_indices + encode_pertinent_payloads over this shard (global indices),
    one RCCL reduce to rank 0, then Retriever::decode_digest on rank 0 (examples/omr.rs:219-293)."""
    import torch

    rp = A.RetrievalParams(total, len(pert))
    n_idx, n_pay, per = rp.max_encode_indices_cipher_count, rp.cmb_cipher_count, rp.cmb_count_per_cipher
    seed = bytes(range(1, 33))
    d_pay = torch.from_numpy(synthetic_payloads(first, D).view(np.int16)).to(dev)
    d_w = torch.from_numpy(A.payload_weights(seed, rp).view(np.int16)).to(dev)
    d_dig = torch.empty((n_idx + n_pay, 2, 2048), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    det.encode_indices_device(d_out.data_ptr(), D, first, total, 9, 0, n_idx, d_dig.data_ptr(), stream.cuda_stream)
    det.encode_payloads_device(d_out.data_ptr(), d_pay.data_ptr(), D, first, total, d_w.data_ptr(), n_pay, per,
                               d_dig[n_idx:].data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if dist:
        dist.reduce(d_dig, dst=0, op=dist.ReduceOp.SUM)  # partial digests (< q2 each), int64 sum
        torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    times = [t1 - t0, t2 - t0]
    if dist:
        tt = torch.tensor(times, dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        times = tt.tolist()
    if rank != 0:
        return None
    digest = d_dig.cpu().numpy().view(np.uint64) % np.uint64(A.Q2)
    t3 = time.perf_counter()
    indices, pays = A.Retriever(rp, pack_a).decode_digest(digest[:n_idx], digest[n_idx:], seed)
    t4 = time.perf_counter()
    ok = indices == [int(v) for v in pert]
    if ok:
        want = np.concatenate([synthetic_payloads(int(i), 1) for i in indices]) if indices else np.zeros((0, 612))
        ok = bool(np.array_equal(pays, want))
    return {"ok": ok, "encode_ms": round(times[0] * 1e3, 2), "encode_reduce_ms": round(times[1] * 1e3, 2),
            "retrieve_ms": round((t4 - t3) * 1e3, 2), "index_ct": n_idx, "payload_ct": n_pay,
            "digest_bytes": int(d_dig.numel() * 8), "collective": "reduce(sum) over RCCL" if dist else "none",
            "pertinent_recovered": len(indices)}


def main():
    args = parse()
    # The JSON line is the only thing on stdout: keep a handle on the real stdout and send fd 1
    # (library chatter, e.g. RCCL's version banner at communicator init) to stderr.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or args.force_dist:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist = None
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    D = args.messages

    # keys + synthetic clues (identical on every rank: seeded, counter-based streams), generated on
    # the GPU (bit-identical to the host generators, tests/test_gpu_parity.py)
    t0 = time.perf_counter()
    pack_a, pack_b = A.SecretKeyPack(42), A.SecretKeyPack(4242)
    cur = torch.cuda.current_stream(dev).cuda_stream
    kbufs = [torch.empty(int(np.prod(shape)), dtype=dt, device=dev)
             for shape, dt in ((A.BSK1_SHAPE, torch.int32), (A.KSK_SHAPE, torch.int32),
                               (A.BSK2_SHAPE, torch.int64), (A.TK_SHAPE, torch.int64))]
    pack_a.generate_detection_key_device(7, *[b.data_ptr() for b in kbufs], stream=cur)
    det = A.Detector.from_device_key(*[b.data_ptr() for b in kbufs], device=local)
    first = rank * D
    total = D * world
    rng = np.random.default_rng(2025)
    pert = np.sort(rng.choice(total, min(args.pertinent, total), replace=False))
    mask = np.zeros(D, dtype=bool)
    mine = pert[(pert >= first) & (pert < first + D)] - first
    mask[mine] = True
    d_ca = torch.empty((D, A.N0), dtype=torch.int16, device=dev)
    d_cb = torch.empty((D, A.CLUE_COUNT), dtype=torch.int16, device=dev)
    d_na, d_nb = torch.empty_like(d_ca), torch.empty_like(d_cb)
    pack_a.gen_clues_device(1000, first, D, d_ca.data_ptr(), d_cb.data_ptr(), stream=cur)
    pack_b.gen_clues_device(1001, first, D, d_na.data_ptr(), d_nb.data_ptr(), stream=cur)
    d_mask = torch.from_numpy(mask).to(dev)[:, None]
    d_ca = torch.where(d_mask, d_ca, d_na).contiguous()
    d_cb = torch.where(d_mask, d_cb, d_nb).contiguous()
    del d_na, d_nb
    torch.cuda.synchronize(dev)
    setup_s = time.perf_counter() - t0

    d_out = torch.empty((D, 2, 2048), dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        det.detect_batch_device(d_ca.data_ptr(), d_cb.data_ptr(), D, d_out.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    det.enable_timing(True)
    stage = {"first_level_ms": 0.0, "key_switch_ms": 0.0, "second_level_ms": 0.0}
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    start.record(stream)
    for i in range(args.steps):
        step()
        info = det.last_timing()  # per-stage HIP events recorded on `stream` (waits for them)
        for k in stage:
            stage[k] += info[k]
        print(f"[bench] rank {rank} step {i + 1}/{args.steps} done", file=sys.stderr, flush=True)
    end.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t
    det.enable_timing(False)
    gpu_ms = start.elapsed_time(end)
    elapsed = max(wall, gpu_ms / 1e3)
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # correctness spot check on this rank's data: the client decrypts (library Retriever, CPU)
    # and every pertinency ciphertext must decode to [1, 0, ..., 0] or all zeros (omd.rs:48-58)
    host = d_out[: min(D, 256)].cpu().numpy().view(np.uint64)
    dec = A.Retriever(A.RetrievalParams(max(1, D), 1), pack_a).decrypt_decode(host)
    ok = bool(np.array_equal(dec[:, 0] == 1, mask[: host.shape[0]]) and not dec[:, 1:].any())

    e2e = None if args.no_e2e else end_to_end(det, pack_a, d_out, D, first, total, pert, dist, dev, stream, rank)

    latency_ms = None
    if not args.no_latency:
        one_out = torch.empty((1, 2, 2048), dtype=torch.int64, device=dev)
        lat = []
        for _ in range(3):
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            det.detect_batch_device(d_ca.data_ptr(), d_cb.data_ptr(), 1, one_out.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize(dev)
            lat.append((time.perf_counter() - t1) * 1e3)
        latency_ms = round(min(lat), 3)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    msgs = args.steps * D * world
    value = msgs / elapsed
    # roofline of the dominant kernel: algorithmic bytes per launch / average launch duration,
    # both from HIP events the library records on `stream` around each launch
    names = A.detect_kernels()
    kms = {"br1": stage["first_level_ms"], "ks": stage["key_switch_ms"], "br2": stage["second_level_ms"]}
    role = max(kms, key=kms.get)
    dom = names[role]
    chunks = -(-D // 16384)
    launches = args.steps * chunks
    avg_launch_s = kms[role] / 1e3 / launches
    per_launch_msgs = D / chunks
    achieved = KERNEL_BYTES[role] * per_launch_msgs / avg_launch_s / 1e9
    pmc = load_profile("pmc_latest.json")
    traffic = None
    if pmc and dom in pmc.get("kernels", {}) and pmc.get("messages_per_launch"):
        traffic = pmc["kernels"][dom]["hbm_bytes_per_launch"] * per_launch_msgs / pmc["messages_per_launch"]
    comp = load_profile("compute_latest.json")
    compute = None
    if comp and dom in comp.get("kernels", {}):
        lane_instr = comp["kernels"][dom]["fp64_lane_instr_per_msg"] * per_launch_msgs / avg_launch_s / 1e12
        flops = comp["kernels"][dom]["fp64_flop_per_msg"] * per_launch_msgs / avg_launch_s / 1e12
        compute = {"bound": "fp64-valu", "kernel": dom, "achieved": round(lane_instr, 2),
                   "peak": round(FP64_PEAK_T_LANE_INSTR, 2), "unit": "T FP64 lane-instr/s",
                   "frac": round(lane_instr / FP64_PEAK_T_LANE_INSTR, 4), "tflops": round(flops, 2),
                   "counts_from": comp.get("source")}
    line = {
        "metric": "detect-phase messages/sec + per-message latency, D=65536 at 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "messages/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / PUBLISHED_CPU_MSG_S, 1),
        "vs_baseline_ref": "published 1-thread AVX-512 CPU detect, 234.07 ms/msg (README.md:122)",
        "dtype": "f64",
        "data": "synthetic (seeded keys and clues; 50 pertinent over the whole job)",
        "config": {"workload": workload_name(D, world),
                   "messages_per_gpu": D, "messages_total": D * world,
                   "pertinent": int(len(pert)), "batch": 16384, "parallelism": f"dp{world}"},
        "latency_ms_per_message": latency_ms,
        "stage_ms_per_step": {k: round(v / args.steps, 2) for k, v in stage.items()},
        "detect_bytes_per_message": DETECT_BYTES,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None if traffic is None else round(traffic),
                     "whole_detect_achieved": round(value / world * DETECT_BYTES / 1e9, 1),
                     "whole_detect_frac": round(value / world * DETECT_BYTES / 1e9 / HBM_PEAK_GBS, 4)},
        "compute": compute,
        "correct": ok,
        "e2e": e2e,
        "setup_s": round(setup_s, 1),
    }
    if not args.no_cpu_baseline and world == 1:
        n = args.cpu_baseline_msgs
        dk = A.DetectionKey(*[b.cpu().numpy().view(np.uint32 if b.dtype == torch.int32 else np.uint64).reshape(shape)
                              for b, shape in zip(kbufs, (A.BSK1_SHAPE, A.KSK_SHAPE, A.BSK2_SHAPE, A.TK_SHAPE))])
        line["cpu_baseline"] = cpu_baseline(dk, d_ca[:n].cpu().numpy().view(np.uint16),
                                            d_cb[:n].cpu().numpy().view(np.uint16), n)
    print(json.dumps(line), file=json_out, flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
