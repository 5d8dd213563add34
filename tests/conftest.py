import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tfhe-omr_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

# PyTorch ships its own copy of the HIP runtime (torch/lib/libamdhip64.so). Loading it before
# libomr_gpu.so makes the library bind to that same copy (soname libamdhip64.so.7); loaded the
# other way round a process ends up with two HIP/HSA runtimes and the second cannot open the
# GPU. Tests that hand torch device buffers to the library rely on this order.
try:
    import torch  # noqa: F401
except ImportError:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU-oracle cases")
