"""Quick device-time probe of the detect pipeline (stage split via HIP events)."""
import sys
import time

sys.path.insert(0, "tests")
import numpy as np  # noqa: E402

import product_lib as PL  # noqa: E402
from product_lib import omr_amd as A  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
a, b, dk = PL.keys()
det = A.Detector(dk)
ca, cb = a.gen_clues(1, 0, D)
det.detect_batch(ca[:256], cb[:256])  # warm
for _ in range(2):
    t = time.time()
    out, info = det.detect_with_time_info(ca, cb)
    wall = time.time() - t
    print(f"D={D} wall={wall:.3f}s device={info['total_ms']:.1f}ms  br1={info['first_level_ms']:.1f} "
          f"ks={info['key_switch_ms']:.1f} br2+trace={info['second_level_ms']:.1f}  "
          f"-> {D / (info['total_ms'] / 1e3):.0f} msg/s (device)", flush=True)
