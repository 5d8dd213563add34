"""Exit-time fault probe: one small detect workload, then a normal exit, to run
under `rocprofv3 --kernel-trace --stats`. Modes:
  thr     chunks on the throughput kernels only (latency threshold 0: no cooperative launches)
  coop    single-message detects on the latency kernels (cooperative two-CU / five-CU launches)
  torch   as coop, with torch imported first (the library then binds torch's bundled HIP runtime)
  reset   as coop, then hipDeviceReset() before the interpreter exits
OMR_COOPERATIVE=0 in the environment makes `coop` run br2l_kernel / trace_kernel instead."""
import ctypes
import sys

mode = sys.argv[1]
if mode == "torch":
    import torch  # noqa: F401
sys.path.insert(0, "tests")
import product_lib as PL  # noqa: E402
from product_lib import omr_amd as A  # noqa: E402

a, b, dk = PL.keys()
det = A.Detector(dk)
ca, cb = a.gen_clues(1000, 0, 16)
if mode == "thr":
    det.set_latency_threshold(0)
for D in (1, 7, 16):
    det.detect_batch(ca[:D], cb[:D])
det.check()
det.close()
if mode == "reset":
    hip = ctypes.CDLL("libamdhip64.so.7")
    print("hipDeviceReset ->", hip.hipDeviceReset(), flush=True)
print(f"{mode}: done", flush=True)
