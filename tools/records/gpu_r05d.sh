#!/bin/bash
# Round 5, call D: br2q variants (LDS accumulator, no W; q2 also output B's keys a digit ahead):
# parity through each variant library, then a same-box A/B with the base build (D = 65,536, twice).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05d
for v in q q2; do
  OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so tools/gpu_step.sh 600 r05d/parity_$v.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exactness.py -x -v --timeout 300 --timeout-method thread -k "real_keys or level2 or edge or high_kappa or structured" || exit 99
  grep -q " passed" gpurun_out/r05d/parity_$v.log && ! grep -q "FAILED\|Error" gpurun_out/r05d/parity_$v.log || { echo "parity failed $v"; exit 98; }
done
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e
cp gpurun_out/bench_variants.log gpurun_out/r05d/
for v in base q q2; do OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 300 python -u tools/l2_occupancy.py >> gpurun_out/r05d/occ.log 2>&1 || exit 97; done
