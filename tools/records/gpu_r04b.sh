# Round-4 variant call: latency variants (br2y: level 2 with the combine/hand-off/inverse split
# over both groups; br1ls: level 1 with the inverse split over four waves; lat2: both) -- parity,
# then a latency A/B; the br2f paired-inverse variant (inv3) -- parity, then a throughput A/B; last
# the exit-time fault capture with /proc/self/maps.
set -o pipefail
out=gpurun_out/r04b
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
lib() { echo $PWD/tfhe-omr_amd/build/var_$1.so; }
for v in br2y br1ls lat2; do
  OMR_GPU_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_exactness.py -x -q -k "latency or real or two_contexts or handoff" --timeout 200 --timeout-method thread > $out/tests_$v.log 2>&1 || exit 4
done
for rep in 1 2; do for v in base br2y br1ls lat2; do
  OMR_GPU_LIB=$(lib $v) timeout -k 10 120 python tools/latency_split.py 1 7 > $out/lat_$v.log 2>&1 && echo "$v $(cat $out/lat_$v.log | tr '\n' ' ')" >> $out/lat_ab.log || exit 5
done; done
OMR_GPU_LIB=$(lib inv3) timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "throughput or small_batches or real" --timeout 150 --timeout-method thread > $out/tests_inv3.log 2>&1 || exit 6
for rep in 1 2; do for v in base inv3; do
  OMR_GPU_LIB=$(lib $v) timeout -k 10 300 python bench.py --messages 16384 --steps 1 --warmup 1 --no-cpu-baseline --no-latency --no-e2e > $out/bv.json 2>> $out/bv.err || exit 7
  echo "$v $(python3 -c "import json;d=json.loads(open('$out/bv.json').readline());print(d['value'],d['ms_per_step'],d['stage_ms_per_step'],d['correct'])")" >> $out/tp_ab.log
done; done
OMR_MAPS_OUT=$out/maps.txt timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -f csv -d $out/kt_latency -o kt -- python tools/latency_split.py 1 7 > $out/latency_prof.log 2>&1
echo "rocprof rc=$?" >> $out/lat_ab.log
