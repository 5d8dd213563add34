#!/bin/bash
# Round 5, call ZI: level 1 (br1f) with one polynomial's digit words live at a time (var_sd: 232
# instead of 250 VGPRs), and with the freed registers holding the first 2 / 4 points' key values
# read before the forward transform's last pass, the row's landing barrier moved there (var_sdek2,
# var_sdek4); level-1 parity through each, then a same-box A/B with var_base = HEAD, twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zi
for v in sd sdek2 sdek4; do
  OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so tools/gpu_step.sh 600 r05zi/tests_$v.log python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread || exit 99
  grep -q "passed" gpurun_out/r05zi/tests_$v.log && ! grep -q "FAILED" gpurun_out/r05zi/tests_$v.log || { echo "tests failed"; exit 98; }
done
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05zi/
