"""bench.py — detect-phase messages/s of the MI355X InstantOMR detector.

Workload: full Detector::detect() (detector.rs:135-166) over synthetic clues (50 pertinent over
the whole job, the rest from a second sender key), inputs resident in HBM, outputs (the
pertinency vector, D x 32 KiB) written to HBM. One step = one detect pass over the clues of
every rank. One process per GPU (torch.distributed, RCCL); each rank owns a contiguous range of
global message indices and detect needs no collective.
  weak scaling (default):  --messages D per GPU (65,536: BASELINE configs[2] at N = 1,
                           configs[3]'s D = 524,288 at N = 8)
  strong scaling:          --total-messages T split over the N GPUs (T = 524,288: configs[3]'s
                           1/2/4/8-GPU curve; T = 2^20: configs[4])

After the timed detect steps, one end-to-end pass (omr_dist.encode_and_reduce, the code path the
gloo test drives) runs on the last pertinency vector: encode_pertinent_indices +
encode_pertinent_payloads over each rank's shard with global indices, one RCCL reduce of the
partial digests to rank 0, and the client-side retrieval (the library's Retriever) must recover
exactly the pertinent indices and their payloads ("e2e"; --no-e2e skips it).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--messages D | --total-messages T]
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
import omr_dist  # noqa: E402

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
# Compulsory HBM bytes: what a detect step must move at least. The device-resident
# key forms are read once per launch: BSK1 FFT form 64 MiB, KSK int8 limbs 84 MiB, BSK2 FFT form
# 503 MiB, trace key 8.6 MiB; per message the clue in, the pertinency ciphertext out and the
# chunk scratch written and read back once (extracted LWEs u32 [7][1025], [1025], [671]).
DEVICE_KEY_BYTES = 512 * 8 * 2 * 512 * 16 + 1024 * 4 * 672 * 32 + 670 * 12 * 4 * 1024 * 16 + 11 * 25 * 2 * 2048 * 8
IO_BYTES_PER_MSG = 512 * 2 + 7 * 2 + 2 * 2048 * 8
SCRATCH_BYTES_PER_MSG = 2 * 4 * (7 * 1025 + 1025 + 671)
DETECT_KERNEL_ROLES = ("br1", "ks", "br2")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
# FP64 VALU peak: 256 CUs x 4 SIMDs x 16 FP64 FMA lanes x 2 FLOP x 2.4 GHz = 78.6 TFLOP/s (a wave64
# FP64 instruction issues in 4 cycles); the arithmetic microbenchmark reaches 95 % of it
# (profiles/r01_microbench_arith.txt).
FP64_PEAK_TFLOPS = 256 * 4 * 16 * 2 * 2.4e9 / 1e12
# L2 -> CU read ceiling: rows every workgroup streams from its XCD's L2, 16 B per lane, 64 KB in
# flight per workgroup, two workgroups per CU: 30.1-30.6 TB/s chip-wide, 118-120 GB/s per CU
# (tools/microbench_l2.hip, profiles/r05o/microbench_l2.log).
L2_CEILING_TBPS = 30.59
# Key bytes each dominant kernel actually reads from L2 per message, in its device form: br2f the
# FFT-form BSK2 (670 steps x 12 rows x 2 outputs x 2 limbs x 1024 points x 16 B; no workgroup
# shares a row), br1f the FFT-form BSK1 rows staged by LDS-DMA once per 4-rotation workgroup.
L2_KEY_BYTES = {"br2": 670 * 12 * 4 * 1024 * 16, "br1": 7 * 512 * 8 * 2 * 512 * 16 // 4}
# Fixed algorithmic FP64 work per message ("fixed-work FLOPs"): a radix-2 complex
# butterfly counts 10 FLOPs (one complex product, two complex additions), an n-point complex FFT
# (n/2) log2 n butterflies, a complex multiply-accumulate 8 FLOPs; rounding, digit extraction and
# recombination count nothing. Constant across rounds: an FMA or tangent-form rewrite of the same
# transforms cannot move it (the counter-based `frac` counts FMA = 2 and can).
#   level 1: 7 rotations x 512 steps x [10 transforms of 512 points (8 digits forward, 2 inverse)
#            + 8 rows x 2 outputs x 512 points MAC]
#   level 2: 670 steps x [16 transforms of 1,024 points (12 digits forward, 4 inverse: 2 outputs x
#            2 key limbs) + 12 rows x 2 outputs x 2 limbs x 1,024 points MAC]
#   trace:   11 automorphisms x [29 transforms of 1,024 points (25 digits, 4 inverse) + 25 rows x
#            2 outputs x 2 limbs x 1,024 points MAC]
FIXED_FLOP_PER_MSG = {
    "br1": 7 * 512 * (10 * (512 // 2) * 9 * 10 + 8 * 2 * 512 * 8),         # 1,060.6 M
    "br2": 670 * (16 * (1024 // 2) * 10 * 10 + 12 * 2 * 2 * 1024 * 8),     #   812.3 M
    "trace": 11 * (29 * (1024 // 2) * 10 * 10 + 25 * 2 * 2 * 1024 * 8),    #    25.3 M
}
PUBLISHED_CPU_MS_PER_MSG = 234.073003  # README.md:122, 1 thread, AVX-512 CPU (model not stated)
WEIGHT_SEED = bytes(range(1, 33))
INDEX_SEED = 9


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--messages", type=int, default=None, help="clues per GPU (weak scaling; default 65,536)")
    g.add_argument("--total-messages", type=int, default=None, help="clues over all GPUs (strong scaling)")
    ap.add_argument("--batch", type=int, default=65536,
                    help="messages per detect launch (omr_ctx_set_batch); 65,536 measured +0.4 %% over 16,384 "
                         "(profiles/r02g/batch_sweep_d65536.log: fewer end-of-launch tails)")
    ap.add_argument("--pertinent", type=int, default=50)
    ap.add_argument("--cpu-single-msgs", type=int, default=8, help="CPU baseline: 1-thread sample")
    ap.add_argument("--cpu-msgs-per-thread", type=int, default=4, help="CPU baseline: all-core sample per thread")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the RCCL process group even at world size 1 (rehearses the N > 1 path)")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal of the N > 1 path on a one-GPU box: every rank uses device 0 and the "
                         "process group is gloo (RCCL cannot run two ranks on one GPU); not a scaling number")
    ap.add_argument("--dist-timeout", type=float, default=120.0,
                    help="seconds before a collective or the rendezvous fails (N > 1): a stuck rank ends the "
                         "run with a non-zero exit instead of a hang")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the encode + reduce + retrieval pass")
    return ap.parse_args()


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> int:
    """Host threads this process may use: its CPU affinity, capped by OMP_NUM_THREADS when set
    (the GPU box exports the box's CPU share there; os.cpu_count() shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(env))) if env.isdigit() and int(env) > 0 else n


def cpu_baseline(dk, ca, cb, single_msgs, per_thread):
    """The oracle detect() (oracle/, plain-C restatement of the reference path: kind "port") timed
    on this host (the Rust reference cannot be built here), per BASELINE.md §3:
    (i) 1 thread, mean over `single_msgs` messages; (ii) every usable core, one message per
    thread at a time like rayon, over per_thread x cores messages. Test infrastructure, used only
    for this reported leg, after the timed GPU region."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    cores = cpu_threads()
    n_all = per_thread * cores
    if ca.shape[0] < max(single_msgs, n_all):
        raise ValueError("not enough clues for the CPU baseline sample")
    det = O.OracleDetector(dk.bsk1, dk.ksk, dk.bsk2, dk.trace_key)
    det.detect_batch(ca[:1], cb[:1], nthreads=1)  # warm the tables
    t = time.perf_counter()
    det.detect_batch(ca[:single_msgs], cb[:single_msgs], nthreads=1)
    t1 = time.perf_counter() - t
    t = time.perf_counter()
    det.detect_batch(ca[:n_all], cb[:n_all], nthreads=cores)
    tn = time.perf_counter() - t
    det.close()
    return {"value": round(n_all / tn, 3), "unit": "messages/s", "cores": cores, "kind": "port",
            "sample": (f"{n_all} detect() calls ({per_thread} per thread) on {cores} threads, OpenMP over "
                       f"messages, {tn:.1f} s wall; 1 thread: {single_msgs} calls, {t1:.1f} s"),
            "single_thread_ms_per_msg": round(t1 / single_msgs * 1e3, 2),
            "all_cores_msgs_per_s": round(n_all / tn, 3),
            "nproc": os.cpu_count(), "cpu_model": cpu_model(),
            "published_reference_ms_per_msg": PUBLISHED_CPU_MS_PER_MSG,
            "published_reference_note": "reference Rust detect(), 1 thread, AVX-512, different machine "
                                        "(README.md:122)"}


def workload_name(per_rank, total, world, strong):
    if strong:
        name = f"full detect() D={total} sharded over {world} GPU(s) (strong scaling)"
        if total == 524288:
            name += " (configs[3])"
        elif total == 1 << 20:
            name += " (configs[4]: detect + encode + retrieval at D=2^20)"
        return name
    name = f"full detect() D={per_rank} per GPU, {total} total (weak scaling)"
    if per_rank == 65536:
        name += " (configs[2] at N=1; configs[3]'s D=524,288 at N=8)"
    elif total == 1 << 20:
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


def rooflines(role, dom, launches, per_launch_msgs, launch_ms_total, value, world, names):
    """Dominant-kernel rooflines from HIP-event launch times and committed counter summaries.
    The blind rotations are VALU-issue and latency bound: `roofline` prices the
    kernel's FP64 FLOPs per launch (counted per message by rocprofv3 SQ_INSTS_VALU_*_F64, FMA = 2)
    against the 78.6 TFLOP/s FP64 peak, and carries the fractions of the VALU issue slots used by
    its FP64 instructions and by all its VALU instructions (the level-2 FFT does 40 % fewer FLOPs
    than round 2's NTT in 6 % less time, so its FLOP fraction is lower). FP64 issue is the binding
    roofline. `hbm` reports HBM honestly: the compulsory bytes of a step and
    the bytes the counters measured (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE), each
    against the 8 TB/s peak, and -- with no fraction, it is not a roofline -- SURVEY.md §8(d)'s
    key-streaming figure (every key byte counted once per message), an effective rate of a batched
    kernel whose concurrent workgroups share every key row through L2."""
    avg_launch_s = launch_ms_total / 1e3 / launches
    pmc, comp = load_profile("pmc_latest.json"), load_profile("compute_latest.json")
    traffic = None
    if pmc and dom in pmc.get("kernels", {}) and pmc.get("messages_per_launch"):
        traffic = pmc["kernels"][dom]["hbm_bytes_per_launch"] * per_launch_msgs / pmc["messages_per_launch"]
    key_stream = KERNEL_BYTES[role] * per_launch_msgs / avg_launch_s / 1e9
    rate = value / world  # messages per second per GPU
    compulsory = DEVICE_KEY_BYTES / per_launch_msgs + IO_BYTES_PER_MSG + SCRATCH_BYTES_PER_MSG  # per message
    step_measured = None
    if pmc and pmc.get("messages_per_launch") and all(names[r] in pmc.get("kernels", {}) for r in DETECT_KERNEL_ROLES):
        step_measured = sum(pmc["kernels"][names[r]]["hbm_bytes_per_launch"] for r in DETECT_KERNEL_ROLES) \
            / pmc["messages_per_launch"] + pmc["kernels"].get("sum7_kernel", {}).get("hbm_bytes_per_launch", 0.0) \
            / pmc["messages_per_launch"]
    hbm = {"binding_roofline": "fp64-valu (DESIGN.md §5): the rotations share every key row through L2",
           "compulsory_bytes_per_msg": round(compulsory),
           "compulsory_GBps": round(compulsory * rate / 1e9, 2),
           "compulsory_frac": round(compulsory * rate / 1e9 / HBM_PEAK_GBS, 5),
           "measured_bytes_per_msg": None if step_measured is None else round(step_measured),
           "measured_GBps": None if step_measured is None else round(step_measured * rate / 1e9, 2),
           "measured_frac": None if step_measured is None else round(step_measured * rate / 1e9 / HBM_PEAK_GBS, 5),
           "dominant_kernel_measured_GBps": None if traffic is None else round(traffic / avg_launch_s / 1e9, 1),
           "key_stream_effective_GBps": round(key_stream, 1),
           "whole_detect_key_stream_effective_GBps": round(rate * DETECT_BYTES / 1e9, 1),
           "key_stream_note": "SURVEY §8(d) model: every key byte counted once per message; an effective rate, "
                              "not HBM traffic (no fraction: it is not bounded by the HBM peak)",
           "measured_from": None if pmc is None else pmc.get("source"),
           "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    roof = None
    if comp and dom in comp.get("kernels", {}):
        k = comp["kernels"][dom]
        tflops = k["fp64_flop_per_msg"] * per_launch_msgs / avg_launch_s / 1e12
        roof = {"bound": "fp64-valu", "kernel": dom, "achieved": round(tflops, 2),
                "peak": round(FP64_PEAK_TFLOPS, 2), "unit": "TFLOP/s", "frac": round(tflops / FP64_PEAK_TFLOPS, 4),
                "traffic": None if traffic is None else round(traffic),
                "avg_launch_ms": round(avg_launch_s * 1e3, 2), "messages_per_launch": per_launch_msgs,
                "fp64_lane_instr_frac": round(k["fp64_lane_instr_per_msg"] * per_launch_msgs / avg_launch_s
                                              / (FP64_PEAK_TFLOPS / 2 * 1e12), 4),
                # every VALU instruction (FP64 or not) takes one issue slot of the same width: the
                # fraction of the chip's VALU issue slots (at 2.4 GHz) the kernel used
                "valu_issue_frac": round(k.get("valu_lane_instr_per_msg", 0.0) * per_launch_msgs / avg_launch_s
                                         / (FP64_PEAK_TFLOPS / 2 * 1e12), 4),
                "counts_from": comp.get("source")}
    if roof is not None and role in FIXED_FLOP_PER_MSG:
        fixed = FIXED_FLOP_PER_MSG[role] * per_launch_msgs / avg_launch_s / 1e12
        roof.update({"fixed_flop_per_msg": FIXED_FLOP_PER_MSG[role], "achieved_fixed_work": round(fixed, 2),
                     "frac_fixed_work": round(fixed / FP64_PEAK_TFLOPS, 4)})
    if roof is not None and role in L2_KEY_BYTES:
        l2 = L2_KEY_BYTES[role] * per_launch_msgs / avg_launch_s / 1e12
        roof["l2_key_stream"] = {"bytes_per_msg": L2_KEY_BYTES[role], "achieved": round(l2, 2),
                                 "ceiling": L2_CEILING_TBPS, "unit": "TB/s", "frac": round(l2 / L2_CEILING_TBPS, 4),
                                 "ceiling_from": "tools/microbench_l2.hip (profiles/r05o/microbench_l2.log)"}
        pk = (pmc or {}).get("kernels", {}).get(dom, {})
        if pk.get("l2_read_bytes_per_launch") and pmc.get("messages_per_launch"):
            # every L1 -> L2 read request of the kernel (TCP_TCC_READ_REQ x 128 B), per message: the
            # key stream plus its twiddle / table / accumulator reads
            mb = pk["l2_read_bytes_per_launch"] / pmc["messages_per_launch"]
            roof["l2_key_stream"].update({"measured_bytes_per_msg": round(mb),
                                          "measured_achieved": round(mb * per_launch_msgs / avg_launch_s / 1e12, 2),
                                          "l2_hit_rate": None if pk.get("l2_hit_rate") is None
                                          else round(pk["l2_hit_rate"], 4),
                                          "measured_from": pmc.get("source")})
    return roof, hbm


def main():
    args = parse()
    # --gpus N without an external launcher (WORLD_SIZE unset): start N ranks here, before anything
    # touches the GPU; rank 0 prints the JSON line. WORLD_SIZE set and != N is an error. The ranks'
    # rendezvous store lives in this process on a port it keeps bound (omr_dist.host_rendezvous).
    try:
        envs = omr_dist.launch_envs(args.gpus, os.environ)
    except ValueError as e:
        print(f"[bench] {e}", file=sys.stderr, flush=True)
        sys.exit(2)
    if envs is not None:
        store = omr_dist.host_rendezvous(envs)
        rc = omr_dist.spawn_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], envs)
        del store
        sys.exit(rc)
    # The JSON line is the only thing on stdout: keep a handle on the real stdout and send fd 1
    # (library chatter, e.g. RCCL's version banner at communicator init) to stderr.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.one_device else int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    if world > 1 or args.force_dist:
        import datetime
        import torch.distributed as dist
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29511"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
        # every collective (and the rendezvous) fails after --dist-timeout seconds instead of hanging
        # until the driver's limit: a stuck or lost rank makes bench.py exit non-zero (for RCCL the
        # blocking wait makes work.wait() raise on the timeout instead of leaving it to the watchdog)
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
        timeout = datetime.timedelta(seconds=args.dist_timeout)
        if args.one_device:
            dist.init_process_group("gloo", timeout=timeout)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=dev, timeout=timeout)
    else:
        dist = None
    if os.environ.get("OMR_BENCH_FAIL_RANK", "") == str(rank):  # test hook: a rank that dies (tests/)
        print(f"[bench] rank {rank} failing on request (OMR_BENCH_FAIL_RANK)", file=sys.stderr, flush=True)
        sys.exit(3)
    if os.environ.get("OMR_BENCH_HANG_RANK", "") == str(rank):  # test hook: a rank that never arrives
        print(f"[bench] rank {rank} hanging on request (OMR_BENCH_HANG_RANK)", file=sys.stderr, flush=True)
        time.sleep(10 * args.dist_timeout + 600)
        sys.exit(4)
    if dist:
        # every rank is up and the group works, before anything expensive; the world size the
        # process group reports goes into the result line (a SCALE record must be what it says)
        dist.barrier()
        world_observed = dist.get_world_size()
        if world_observed != world:
            raise RuntimeError(f"process group has {world_observed} ranks, WORLD_SIZE={world}")
    else:
        world_observed = 1
    torch.cuda.set_device(local)
    strong = args.total_messages is not None
    if strong:
        first, D, total = omr_dist.plan(rank, world, total=args.total_messages)
    else:
        first, D, total = omr_dist.plan(rank, world, per_gpu=args.messages or 65536)

    # keys + synthetic clues (identical on every rank: seeded, counter-based streams), generated on
    # the GPU (bit-identical to the host generators and the oracle's)
    t0 = time.perf_counter()
    pack_a, pack_b = A.SecretKeyPack(42), A.SecretKeyPack(4242)
    cur = torch.cuda.current_stream(dev).cuda_stream
    kbufs = [torch.empty(int(np.prod(shape)), dtype=dt, device=dev)
             for shape, dt in ((A.BSK1_SHAPE, torch.int32), (A.KSK_SHAPE, torch.int32),
                               (A.BSK2_SHAPE, torch.int64), (A.TK_SHAPE, torch.int64))]
    pack_a.generate_detection_key_device(7, *[b.data_ptr() for b in kbufs], stream=cur)
    det = A.Detector.from_device_key(*[b.data_ptr() for b in kbufs], device=local)
    det.set_batch(args.batch)
    rng = np.random.default_rng(2025)
    pert = np.sort(rng.choice(total, min(args.pertinent, total), replace=False))
    mask = np.zeros(D, dtype=bool)
    mask[pert[(pert >= first) & (pert < first + D)] - first] = True
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

    stream = torch.cuda.current_stream(dev)
    backend = omr_dist.GpuBackend(det, dev, stream)
    d_out = torch.empty((D, 2, 2048), dtype=torch.int64, device=dev)

    for _ in range(args.warmup):
        backend.detect(d_ca, d_cb, out=d_out)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    det.enable_timing(1)  # stage events around the production kernels (trace fused into level 2)
    stage = {"first_level_ms": 0.0, "key_switch_ms": 0.0, "second_level_ms": 0.0, "trace_ms": 0.0}
    per_step = {"first_level_ms": [], "second_level_ms": [], "step_ms": []}
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    start.record(stream)
    for i in range(args.steps):
        ts = time.perf_counter()
        backend.detect(d_ca, d_cb, out=d_out)
        info = det.last_timing()  # per-stage HIP events recorded on `stream` (waits for them)
        per_step["step_ms"].append((time.perf_counter() - ts) * 1e3)
        for k in stage:
            stage[k] += info[k]
        per_step["first_level_ms"].append(info["first_level_ms"] - info["key_switch_ms"])
        per_step["second_level_ms"].append(info["second_level_ms"])
        print(f"[bench] rank {rank} step {i + 1}/{args.steps} done", file=sys.stderr, flush=True)
    end.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t
    backend.synchronize()  # raises if a detect call failed on the device
    gpu_ms = start.elapsed_time(end)
    elapsed = max(wall, gpu_ms / 1e3)
    rank_elapsed = [elapsed]
    if dist:
        # every rank's timed region, gathered (the line reports the spread); the value uses the max
        tt = torch.zeros(world_observed, dtype=torch.float64, device=dev)
        tt[rank] = elapsed
        tt = omr_dist._on_backend(tt, dist)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        rank_elapsed = [float(v) for v in tt.tolist()]
        elapsed = max(rank_elapsed)

    # Detector::detect_with_time_info's split (detector.rs:169-221) on one untimed pass: timing
    # mode 2 runs the level-2 rotation and the trace as two launches, so the trace gets its own time
    det.enable_timing(2)
    backend.detect(d_ca, d_cb, out=d_out)
    split = det.last_timing()
    det.enable_timing(0)
    backend.synchronize()
    time_info = {"total_detect_ms": round(split["total_ms"], 2),
                 "first_level_bootstrapping_ms": round(split["first_level_ms"], 2),
                 "second_level_bootstrapping_ms": round(split["second_level_ms"], 2),
                 "trace_ms": round(split["trace_ms"], 2),
                 "key_switch_ms": round(split["key_switch_ms"], 2), "messages": int(split["messages"]),
                 "trace_separate": bool(split["trace_separate"]),
                 "note": "one untimed detect pass in timing mode 2 (trace as its own launch); DetectTimeInfo "
                         "fields (detector.rs:51-57), first level includes the key switch"}

    # Exactness certificate of the FFT external products on this run's clues: one
    # untimed pass through the guarded kernels records the largest |y - rint(y)| of every rounded
    # coefficient; with the key's a priori bound E the run is exact when margin < 1 - E. The pass runs
    # in slices of at most one launch (--batch), each compared with the timed output: the extra
    # device memory is one slice whatever D is.
    det.rounding_margin(reset=True)
    det.set_rounding_guard(True)
    G = min(D, args.batch)
    g_out = torch.empty((G, 2, 2048), dtype=torch.int64, device=dev)
    identical = True
    guarded_ms = 0.0
    for s0 in range(0, D, G):
        n = min(G, D - s0)
        torch.cuda.synchronize(dev)
        tg = time.perf_counter()
        det.detect_batch_device(d_ca[s0:].data_ptr(), d_cb[s0:].data_ptr(), n, g_out.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        guarded_ms += (time.perf_counter() - tg) * 1e3
        identical &= bool(torch.equal(g_out[:n], d_out[s0:s0 + n]))
    det.set_rounding_guard(False)
    backend.synchronize()
    del g_out
    rm = det.rounding_margin(reset=True)
    ex = det.exactness()
    exactness = {"observed_margin": [float(f"{v:.4g}") for v in rm["observed"]],
                 "apriori_bound": [round(v, 4) for v in rm["apriori"]],
                 "certified": all(o < 1 - e for o, e in zip(rm["observed"], rm["apriori"])),
                 "guarded_output_identical": identical,
                 "guarded_every_launch": ex["guarded"], "breaches": ex["breaches"],
                 # what a key with E >= 0.5 (guarded on every launch, exactness contract) would cost:
                 # the same detect through the guarded kernels + their no-op fallbacks + the folds
                 "guarded_ms_per_step": round(guarded_ms, 1),
                 "guarded_over_timed": round(guarded_ms / (elapsed / args.steps * 1e3), 4),
                 "note": "level 1, level 2: largest |y - rint(y)| over every rounded FFT product coefficient "
                         "of one untimed guarded pass; exact when observed < 1 - apriori (DESIGN.md §3a); a "
                         "level with apriori >= 0.5 would be guarded on every launch (omr_ctx_exactness)"}

    # correctness spot check on this rank's data: the client decrypts (library Retriever, CPU)
    # and every pertinency ciphertext must decode to [1, 0, ..., 0] or all zeros (omd.rs:48-58)
    host = d_out[: min(D, 256)].cpu().numpy().view(np.uint64)
    dec = A.Retriever(A.RetrievalParams(max(1, total), 1), pack_a).decrypt_decode(host)
    ok = bool(np.array_equal(dec[:, 0] == 1, mask[: host.shape[0]]) and not dec[:, 1:].any())

    e2e = None
    if not args.no_e2e:
        rp = A.RetrievalParams(total, len(pert))
        weights = A.payload_weights(WEIGHT_SEED, rp)
        digest, et = omr_dist.encode_and_reduce(backend, d_out, synthetic_payloads(first, D), first, total, rp,
                                                INDEX_SEED, weights, dist)
        if rank == 0:
            t3 = time.perf_counter()
            indices, pays = A.Retriever(rp, pack_a).decode_digest(digest.indices, digest.payloads, WEIGHT_SEED)
            t4 = time.perf_counter()
            good = indices == [int(v) for v in pert]
            if good:
                want = np.concatenate([synthetic_payloads(int(i), 1) for i in indices]) if indices else np.zeros((0, 612))
                good = bool(np.array_equal(pays, want))
            e2e = {"ok": good, "encode_ms": round(et["encode_s"] * 1e3, 2),
                   "encode_reduce_ms": round(et["encode_reduce_s"] * 1e3, 2), "retrieve_ms": round((t4 - t3) * 1e3, 2),
                   "index_ct": rp.max_encode_indices_cipher_count, "payload_ct": rp.cmb_cipher_count,
                   "digest_bytes": int((rp.max_encode_indices_cipher_count + rp.cmb_cipher_count) * 2 * 2048 * 8),
                   "collective": "reduce(sum) over RCCL" if dist else "none", "pertinent_recovered": len(indices)}

    latency_ms = latency_tp_ms = None
    if not args.no_latency:
        # one message end to end (detect on device buffers, wall clock): the latency kernels
        # (default for chunks up to 64 messages) and, for comparison, the throughput kernels
        one_out = torch.empty((1, 2, 2048), dtype=torch.int64, device=dev)

        def one_message():
            lat = []
            for _ in range(3):
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                det.detect_batch_device(d_ca.data_ptr(), d_cb.data_ptr(), 1, one_out.data_ptr(), stream.cuda_stream)
                torch.cuda.synchronize(dev)
                lat.append((time.perf_counter() - t1) * 1e3)
                det.check(stream.cuda_stream)  # raises on a failed two-CU hand-off
                if not torch.equal(one_out[0], d_out[0]):  # same message as the timed throughput pass
                    raise RuntimeError("single-message detect differs from the throughput kernels' output")
            return round(min(lat), 3)

        latency_ms = one_message()
        det.set_latency_threshold(0)
        latency_tp_ms = one_message()
        det.set_latency_threshold(64)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    msgs = args.steps * total
    value = msgs / elapsed
    names = A.detect_kernels()
    # per-kernel launch times: level 2's rotation (br2f_kernel) and its trace (trace_fft_kernel) are
    # separate launches since round 5, so the rotation's time is second_level alone
    kms = {"br1": stage["first_level_ms"] - stage["key_switch_ms"], "ks": stage["key_switch_ms"],
           "br2": stage["second_level_ms"]}
    role = max(kms, key=kms.get)
    chunks = -(-D // args.batch)
    roof, hbm = rooflines(role, names[role], args.steps * chunks, D / chunks, kms[role], value, world, names)
    # the other blind rotation's roofline the same way (its own live launch time and counted FLOPs)
    other_roofs = {}
    for r in ("br1", "br2"):
        if r != role:
            ro, _ = rooflines(r, names[r], args.steps * chunks, D / chunks, kms[r], value, world, names)
            if ro is not None:
                other_roofs[r] = ro
    # whole-detect FP64 fractions: counted FLOPs (profiles/compute_latest.json, FMA = 2) and the fixed
    # algorithmic FLOPs (FIXED_FLOP_PER_MSG), both at the whole job's per-GPU rate
    comp = load_profile("compute_latest.json") or {}
    ck = comp.get("kernels", {})
    counted = sum(ck.get(n, {}).get("fp64_flop_per_msg", 0.0) for n in (names["br1"], names["br2"], "trace_fft_kernel"))
    rate = value / world
    detect_fp64 = {"counted_flop_per_msg": round(counted), "fixed_flop_per_msg": sum(FIXED_FLOP_PER_MSG.values()),
                   "detect_fp64_frac": round(counted * rate / 1e12 / FP64_PEAK_TFLOPS, 4) if counted else None,
                   "detect_fp64_frac_fixed_work": round(sum(FIXED_FLOP_PER_MSG.values()) * rate / 1e12
                                                        / FP64_PEAK_TFLOPS, 4),
                   "peak_tflops": round(FP64_PEAK_TFLOPS, 2), "counts_from": comp.get("source"),
                   "note": "FP64 FLOPs of the whole detect (both rotations + the FFT trace) per message x the "
                           "per-GPU msg/s over the FP64 peak; fixed_work: the constant algorithmic count of "
                           "DESIGN.md §5 (10 FLOPs per radix-2 butterfly, 8 per complex MAC)"}

    def spread(v):
        v = sorted(v)
        return {"min": round(v[0], 2), "median": round(float(np.median(v)), 2), "max": round(v[-1], 2),
                "max_over_min": round(v[-1] / v[0], 4) if v[0] > 0 else None}

    line = {
        "metric": "detect-phase messages/sec + per-message latency, D=65536 at 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "messages/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": round(value / (1e3 / PUBLISHED_CPU_MS_PER_MSG), 1),
        "vs_baseline_ref": "published reference detect(), 1 thread AVX-512 CPU, 234.07 ms/msg at D=65,536 "
                           "(README.md:122, BASELINE.md §1)",
        "dtype": "f64",
        "data": "synthetic (seeded keys and clues generated on the GPU; 50 pertinent over the whole job)",
        "config": {"workload": workload_name(D, total, world, strong),
                   "messages_per_gpu": D, "messages_total": total,
                   "pertinent": int(len(pert)), "batch": args.batch, "parallelism": f"dp{world}"},
        "latency_ms_per_message": latency_ms,
        "latency_ms_per_message_throughput_kernels": latency_tp_ms,
        "stage_ms_per_step": dict({k: round(v / args.steps, 2) for k, v in stage.items()},
                                  note="timed steps: first_level includes the key switch; second_level is the "
                                       "level-2 rotation (br2f_kernel), trace the FFT trace's own launch "
                                       "(trace_fft_kernel)"),
        "per_step_spread": {"level1_rotation_ms": spread(per_step["first_level_ms"]),
                            "level2_rotation_ms": spread(per_step["second_level_ms"]),
                            "step_wall_ms": spread(per_step["step_ms"]),
                            "note": "rank 0, over the K timed steps: level1 = br1f_kernel (first level minus the key "
                                    "switch), level2 = br2f_kernel, from the stage HIP events; step_wall = host "
                                    "wall clock of one detect call"},
        "dist": {"world_size_observed": world_observed, "backend": dist.get_backend() if dist else None,
                 "rank_elapsed_s": {"min": round(min(rank_elapsed), 3), "max": round(max(rank_elapsed), 3)},
                 "timeout_s": args.dist_timeout if dist else None},
        "detect_fp64": detect_fp64,
        "detect_time_info": time_info,
        "detect_bytes_per_message": DETECT_BYTES,
        "roofline": roof,
        "roofline_other_rotation": other_roofs or None,
        "hbm": hbm,
        "correct": ok,
        "exactness": exactness,
        "e2e": e2e,
        "setup_s": round(setup_s, 1),
    }
    if not args.no_cpu_baseline and world == 1:
        n = max(args.cpu_single_msgs, args.cpu_msgs_per_thread * cpu_threads())
        dk = A.DetectionKey(*[b.cpu().numpy().view(np.uint32 if b.dtype == torch.int32 else np.uint64).reshape(shape)
                              for b, shape in zip(kbufs, (A.BSK1_SHAPE, A.KSK_SHAPE, A.BSK2_SHAPE, A.TK_SHAPE))])
        ca, cb = pack_a.gen_clues(1000, 0, n)  # the same clue stream as the GPU workload
        line["cpu_baseline"] = cpu_baseline(dk, ca, cb, args.cpu_single_msgs, args.cpu_msgs_per_thread)
    print(json.dumps(line), file=json_out, flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
