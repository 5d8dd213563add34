"""Per-phase durations of the latency kernels from a -DOMR_PHASE_TRACE build
(tools/build_variant.sh phase -DOMR_PHASE_TRACE; OMR_GPU_LIB=.../var_phase.so python tools/phase_trace.py).
Runs one single-message detect (latency path) and prints the mean cycles between consecutive phase
marks of executed steps 200..263 for every traced wave (br1l workgroup 0; br2x workgroups 0, 1)."""
import ctypes
import os
import sys

sys.path.insert(0, "tests")
import numpy as np  # noqa: E402

import product_lib as PL  # noqa: E402
from product_lib import omr_amd as A  # noqa: E402

PT_STEPS, PT_K, PT_SLOTS = 64, 8, 32
a, b, dk = PL.keys()
det = A.Detector(dk)
ca, cb = a.gen_clues(1000, 0, 256)
det.detect_batch(ca[:1], cb[:1])
det.detect_batch(ca[1:2], cb[1:2])
n = PT_SLOTS * PT_STEPS * PT_K + PT_SLOTS * 4
buf = (ctypes.c_ulonglong * n)()
lib = A.lib()
lib.omr_debug_phase_read.restype = ctypes.c_int
got = lib.omr_debug_phase_read(buf, ctypes.c_size_t(n))
assert got == n, got
arr = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
marks = arr[: PT_SLOTS * PT_STEPS * PT_K].reshape(PT_SLOTS, PT_STEPS, PT_K)
clk = arr[PT_SLOTS * PT_STEPS * PT_K:].reshape(PT_SLOTS, 4)
names = {  # phase ending at mark k (k = 1..7); br2x has no mark 2 (a mark there makes it spill)
    "br1l": {1: "digits", 2: "fwd + spectrum store", 3: "barrier1", 4: "mac + stores + barrier2",
             5: "outs read", 6: "inverse", 7: "update + barrier3"},
    "br2x": {1: "stage+digits", 3: "3 fwd + MAC + g1 partial + barrier", 4: "g0 sum + sc1 stores + vmcnt + barrier",
             5: "flag + poll + barrier", 6: "sc1 loads + inverse (g0) / barrier (g1)", 7: "update"},
    "br2y": {1: "barrier + digits", 2: "3 fwd + MAC", 3: "limb-swap writes + barrier",
             4: "sums + sc1 stores + vmcnt + barrier", 5: "flag + poll + barrier", 6: "sc1 loads + inverse",
             7: "round + half swap + barrier + update"},
}
for slot in range(24):
    kern = "br1l" if slot < 8 else ("br2x" if os.environ.get("OMR_BR2Y") == "0" else "br2y")
    m = marks[slot]
    if not m[:, 0].any():
        continue
    c0, w0, c1, w1 = clk[slot]
    mhz = (c1 - c0) / ((w1 - w0) / 100.0) if w1 > w0 else float("nan")
    step = np.diff(m[:, 0]).mean() if PT_STEPS > 1 else 0
    present = [k for k in range(PT_K) if m[:, k].all()]  # marks this wave records
    parts = "  ".join(f"{names[kern].get(k1, f'->{k1}')} {(m[:, k1] - m[:, k0]).mean():.0f}"
                      for k0, k1 in zip(present, present[1:]))
    lab = f"{kern} wg{(slot - 8) // 8 if slot >= 8 else 0} wave{slot % 8}"
    print(f"{lab}: clock {mhz:.0f} MHz, step {step:.0f} cyc ({step / mhz:.2f} us) | {parts}", flush=True)
det.close()
