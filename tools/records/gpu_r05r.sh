#!/bin/bash
# Round 5, call R: level-1 P0 <-> P1 relayout through the wave's LDS buffer instead of 32 permlanes
# per transform (-DOMR_BR1_X01) -- level-1 parity through the variant, then a same-box A/B twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05r
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_x01.so tools/gpu_step.sh 300 r05r/parity_x01.log python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "fft1 or level1 or real_keys or edge" || exit 99
grep -q "passed" gpurun_out/r05r/parity_x01.log && ! grep -q "FAILED" gpurun_out/r05r/parity_x01.log || { echo "parity failed"; exit 98; }
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05r/
