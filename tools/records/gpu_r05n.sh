#!/bin/bash
# Round 5, call N: level-2 digit words from the FP64 bit pattern + the one-quotient limb update,
# level-1 unshifted digit words -- the GPU suite on the new library, then a same-box A/B (var_base =
# the previous HEAD, var_new = this library, var_sh = var_new with the shifted level-1 words) twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05n
tools/gpu_step.sh 600 r05n/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05n/gpu_tests.log && ! grep -q "FAILED" gpurun_out/r05n/gpu_tests.log || { echo "suite failed"; exit 98; }
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05n/
