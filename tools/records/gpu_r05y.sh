#!/bin/bash
# Round 5, call Y: level 2's trace as its own launch on the FFT (trace_fft_kernel) and the closed-form
# trace digits -- the full GPU suite on the new library, then a same-box A/B (var_base = the previous
# library with the fused NTT trace, var_tr = this one) twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05y
tools/gpu_step.sh 700 r05y/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05y/gpu_tests.log && ! grep -q "FAILED" gpurun_out/r05y/gpu_tests.log || { echo "suite failed"; exit 98; }
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05y/
