#!/bin/bash
# Round 5, call J: tangent-form level-1 forward butterflies -- the full GPU suite (parity, exactness,
# guard margins), then a same-box A/B against the previous library (var_base) twice, then the
# default bench line.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05j
tools/gpu_step.sh 1000 r05j/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05j/gpu_tests.log && ! grep -q "FAILED" gpurun_out/r05j/gpu_tests.log || { echo "suite failed"; exit 98; }
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05j/
tools/gpu_step.sh 600 r05j/bench.log python bench.py || exit 99
