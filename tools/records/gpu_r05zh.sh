#!/bin/bash
# Round 5, call ZH: var_kbs = br2f's output-B limb-0 key blocks issued before the digit's forward
# transform (instead of after its cross-wave exchange); parity through it, then a same-box A/B with
# var_base = HEAD, twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zh
for v in kbs; do
  OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so tools/gpu_step.sh 600 r05zh/tests_$v.log python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread || exit 99
  grep -q "passed" gpurun_out/r05zh/tests_$v.log && ! grep -q "FAILED" gpurun_out/r05zh/tests_$v.log || { echo "tests failed"; exit 98; }
done
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05zh/
