"""bench.py — detect-phase messages/s of the MI355X InstantOMR detector.

Workload (BASELINE.json configs[2]): full Detector::detect() (detector.rs:135-166) over
D = 65,536 synthetic clues per GPU (50 pertinent, the rest from a second sender key),
inputs resident in HBM, outputs (the pertinency vector, D x 32 KiB) written to HBM.
One step = one detect pass over the D clues of every rank. N > 1: one process per GPU
(torch.distributed, RCCL), each rank owns a contiguous range of global message indices
(weak scaling, no data-path collective). Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--messages D]
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
KERNEL_BYTES = {  # per message, per kernel of the pipeline
    "br1_kernel": BR1_BYTES + 7 * (512 * 2 + 2) + 7 * 1025 * 4,
    "ks_kernel": KS_BYTES + 1025 * 4 + 671 * 4,
    "br2_trace_kernel": BR2_BYTES + TRACE_BYTES + 671 * 4 + 2 * 2048 * 8,
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
PUBLISHED_CPU_MSG_S = 1e3 / 234.073003  # README.md:122, 1 thread AVX-512


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--messages", type=int, default=65536, help="clues per GPU")
    ap.add_argument("--pertinent", type=int, default=50)
    ap.add_argument("--cpu-baseline-msgs", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
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


def load_pmc_traffic():
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (profiles/*pmc*.json, produced by tools/profile.sh on the GPU box), else None."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("kernel"), d


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist = None
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    D = args.messages

    # keys + synthetic clues (identical on every rank: seeded, counter-based streams)
    t0 = time.perf_counter()
    pack_a, pack_b = A.SecretKeyPack(42), A.SecretKeyPack(4242)
    dk = pack_a.generate_detection_key(7)
    first = rank * D
    total = D * world
    rng = np.random.default_rng(2025)
    pert = np.sort(rng.choice(total, min(args.pertinent, total), replace=False))
    mask = np.zeros(D, dtype=bool)
    mine = pert[(pert >= first) & (pert < first + D)] - first
    mask[mine] = True
    ca, cb = pack_a.gen_clues(1000, first, D)
    na, nb = pack_b.gen_clues(1001, first, D)
    ca[~mask], cb[~mask] = na[~mask], nb[~mask]
    det = A.Detector(dk, device=local)
    setup_s = time.perf_counter() - t0

    d_ca = torch.from_numpy(ca.view(np.int16)).to(dev)
    d_cb = torch.from_numpy(cb.view(np.int16)).to(dev)
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
    for _ in range(args.steps):
        step()
        info = det.last_timing()  # per-stage HIP events recorded on `stream`
        for k in stage:
            stage[k] += info[k]
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

    # correctness spot check on this rank's data (device result, client-side decrypt)
    ok = True
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import retriever as R
        s2 = pack_a.export()["s2"]
        host = d_out[: min(D, 256)].cpu().numpy().view(np.uint64)
        for m in range(host.shape[0]):
            dec = R.decrypt_decode(s2, host[m])
            ok &= bool((dec[0] == 1) == mask[m]) and not dec[1:].any()
    except Exception as e:  # noqa: BLE001
        ok = f"check failed: {e}"

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
    # roofline of the dominant kernel: algorithmic bytes per launch / average launch duration
    kms = {"br1_kernel": stage["first_level_ms"], "ks_kernel": stage["key_switch_ms"],
           "br2_trace_kernel": stage["second_level_ms"]}
    dom = max(kms, key=kms.get)
    chunks = -(-D // 16384)
    launches = args.steps * chunks
    avg_launch_s = kms[dom] / 1e3 / launches
    per_launch_msgs = D / chunks
    achieved = KERNEL_BYTES[dom] * per_launch_msgs / avg_launch_s / 1e9
    pmc_kernel, pmc = load_pmc_traffic()
    traffic = None
    if pmc and pmc_kernel == dom and pmc.get("messages_per_launch"):
        traffic = pmc["hbm_bytes_per_launch"] * per_launch_msgs / pmc["messages_per_launch"]
    line = {
        "metric": "detect-phase messages/sec (D=65536 per GPU)",
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
        "config": {"workload": "full detect() D=65536 per GPU (configs[2]; configs[3] at N=8)",
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
        "correct": ok,
        "setup_s": round(setup_s, 1),
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(dk, ca, cb, args.cpu_baseline_msgs)
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
