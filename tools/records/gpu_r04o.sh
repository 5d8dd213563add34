# In-wave LDS exchanges without the lgkmcnt(0) park (OMR_LDS_INORDER=1): the full GPU suite on the
# variant library, then base vs inorder timing twice and single-message latency.
# (Record of a round-4 A/B: the var_*.so it times were built by tools/build_variant.sh from scratch
# edits / -D switches that were folded into or removed from the sources afterwards)
set -o pipefail
out=gpurun_out/r04o
mkdir -p $out
rm -f gpurun_out/bench_variants.log
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_inorder.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/gpu_tests_inorder.log 2>&1 || exit 1
tools/bench_variants.sh 16384 --no-e2e || exit 2
tools/bench_variants.sh 16384 --no-e2e || exit 3
cp gpurun_out/bench_variants.log $out/ab.log
for v in base inorder base inorder; do OMR_KEEP_DEVICE=1 OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 120 python tools/latency_split.py 1 7 > $out/lat_$v.log 2>&1 && echo "$v $(cat $out/lat_$v.log | tr '\n' ' ')" >> $out/lat_ab.log || exit 5; done
