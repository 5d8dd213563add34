# br1f pass-3 twiddles held in registers (OMR_BR1_W3REG): base vs w3, three times each; the parity
# tests of the level-1 paths on w3.
# (Record of a round-4 A/B: the var_*.so it times were built by tools/build_variant.sh from scratch
# edits / -D switches that were folded into or removed from the sources afterwards)
set -o pipefail
out=gpurun_out/r04p
mkdir -p $out
rm -f gpurun_out/bench_variants.log
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_w3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exactness.py -x -q --timeout 500 --timeout-method thread > $out/gpu_tests_w3.log 2>&1 || exit 1
for i in 1 2 3; do tools/bench_variants.sh 16384 --no-e2e || exit 2; done
cp gpurun_out/bench_variants.log $out/ab.log
