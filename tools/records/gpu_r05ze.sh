#!/bin/bash
# Round 5, call ZE: level 1 with one workgroup barrier per key row (br1f_row under OMR_BR1_ONE_BARRIER:
# row q + 1's LDS-DMA issued after row q's landing barrier instead of behind a second barrier) --
# the level-1 parity tests through the variant, then a same-box A/B (var_base = HEAD, var_b1) twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ze
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_b1.so tools/gpu_step.sh 600 r05ze/tests_b1.log python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05ze/tests_b1.log && ! grep -q "FAILED" gpurun_out/r05ze/tests_b1.log || { echo "tests failed"; exit 98; }
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05ze/
