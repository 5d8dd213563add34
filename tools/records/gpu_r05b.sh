#!/bin/bash
# Round 5, call B: level-2 pipelined kernel (br2p, OMR_BR2_PIPE=1) -- parity through the variant
# library, then a same-box A/B against the base build (bench.py, D = 65,536, twice each).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05b
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_pipe.so tools/gpu_step.sh 600 r05b/parity_pipe.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exactness.py -x -v --timeout 300 --timeout-method thread -k "not full_launch" || exit 99
grep -q " passed" gpurun_out/r05b/parity_pipe.log && ! grep -q "FAILED\|Error" gpurun_out/r05b/parity_pipe.log || { echo "parity failed"; exit 98; }
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e
cp gpurun_out/bench_variants.log gpurun_out/r05b/
