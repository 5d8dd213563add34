# Next pass's twiddles read with each LDS exchange (Fft512 pass 2 / inverse pass 1: OMR_FFT1_TWX;
# Fft1024 passes 2, 4 / inverse 3, 1: OMR_BR2_TWX): full GPU suite on twx, then base / twx /
# level-1 only / level-2 only, twice.
# (Record of a round-4 A/B: the var_*.so it times were built by tools/build_variant.sh from scratch
# edits / -D switches that were folded into or removed from the sources afterwards)
set -o pipefail
out=gpurun_out/r04u
mkdir -p $out
rm -f gpurun_out/bench_variants.log
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_twx.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/gpu_tests_twx.log 2>&1 || exit 1
tools/bench_variants.sh 16384 --no-e2e || exit 2
tools/bench_variants.sh 16384 --no-e2e || exit 3
cp gpurun_out/bench_variants.log $out/ab.log
