#!/bin/bash
# Round 5: level 1 on the exact modular NTT (br1_ntt.hpp) -- the level-1 breach fallback, the
# set_exact_level1 cross-check at oracle sizes and at D = 65,536.
set -o pipefail
mkdir -p gpurun_out/r05za
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_exactness.py \
  -k "exact_level1 or high_kappa" > gpurun_out/r05za/tests.log 2>&1
rc=$?; tail -15 gpurun_out/r05za/tests.log; exit $rc
