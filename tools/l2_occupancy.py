"""Level-2 throughput-kernel time vs batch size (diagnoses workgroups per CU): omr_blind_rotate_level2
on n random LWEs with the latency threshold at 0, device time by wall clock around the call (the
copies are < 5 % at these sizes). Library variant via OMR_GPU_LIB. python tools/l2_occupancy.py"""
import os
import sys
import time

sys.path.insert(0, "tests")
import numpy as np  # noqa: E402

import product_lib as PL  # noqa: E402
from product_lib import omr_amd as A  # noqa: E402

_, _, dk = PL.keys()
det = A.Detector(dk)
det.set_latency_threshold(0)
name = os.path.basename(os.environ.get("OMR_GPU_LIB", "libomr_gpu.so"))
rng = np.random.default_rng(1)
for n in (256, 512, 768, 1024, 2048):
    x = rng.integers(0, 4096, size=(n, A.NI + 1), dtype=np.uint32)
    det.blind_rotate_level2(x[:8])
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        det.blind_rotate_level2(x)
        best = min(best, time.perf_counter() - t)
    print(f"{name} n={n}: {best * 1e3:.1f} ms, {best * 1e6 / n:.1f} us/msg", flush=True)
det.close()
