# Round-4 validation call: exactness + coalescing tests, full GPU suite, bench, the br2y latency
# variant (parity + A/B), throughput variant A/B, then the exit-time fault capture (last).
set -o pipefail
out=gpurun_out/r04a
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 python -u -m pytest tests/test_gpu_exactness.py tests/test_gpu_coalesce.py -x -v -s --timeout 400 --timeout-method thread > $out/exact.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || exit 3
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_br2y.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q -k "latency or real or two_contexts" --timeout 200 --timeout-method thread > $out/br2y_tests.log 2>&1 || exit 4
for v in base br2y base br2y; do OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 120 python tools/latency_split.py 1 7 > $out/lat_$v.log 2>&1 && echo "$v $(cat $out/lat_$v.log | tr '\n' ' ')" >> $out/lat_ab.log || exit 5; done
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_inv3.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "throughput or small_batches or real" --timeout 150 --timeout-method thread > $out/inv3_tests.log 2>&1 || exit 6
tools/bench_variants.sh 16384 --no-e2e || exit 7
tools/bench_variants.sh 16384 --no-e2e || exit 8
OMR_MAPS_OUT=$out/maps.txt timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -f csv -d $out/kt_latency -o kt -- python tools/latency_split.py 1 7 > $out/latency_prof.log 2>&1
echo "rocprof rc=$?" >> $out/lat_ab.log
