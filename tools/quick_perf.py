"""Quick device-time probe of the detect pipeline (stage split via HIP events) + output hash.
Library variant via OMR_GPU_LIB. Usage: python tools/quick_perf.py [D] [reps]"""
import hashlib
import os
import sys
import time

sys.path.insert(0, "tests")
import numpy as np  # noqa: E402

import product_lib as PL  # noqa: E402
from product_lib import omr_amd as A  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
a, b, dk = PL.keys()
det = A.Detector(dk)
ca, cb = a.gen_clues(1, 0, D)
det.detect_batch(ca[:256], cb[:256])  # warm
name = os.path.basename(os.environ.get("OMR_GPU_LIB", "libomr_gpu.so"))
for _ in range(reps):
    t = time.time()
    out, info = det.detect_with_time_info(ca, cb)
    wall = time.time() - t
    h = hashlib.sha256(out.tobytes()).hexdigest()[:16]
    print(f"{name:22s} D={D} device={info['total_ms']:.1f}ms br1={info['first_level_ms']:.1f} "
          f"ks={info['key_switch_ms']:.1f} br2+trace={info['second_level_ms']:.1f} "
          f"-> {D / (info['total_ms'] / 1e3):.0f} msg/s  sha={h}", flush=True)
