#!/bin/bash
# Round 5, call I: beyond-L2 traffic (FETCH_SIZE) of level 2 at D = 65,536 for the HEAD library and
# the hand-scheduled br2s variant (does the slowdown at scale come from key-row L2 misses?).
export TMPDIR=/tmp
out=gpurun_out/r05i
mkdir -p $out
B="bench.py --steps 1 --warmup 0 --messages 65536 --no-cpu-baseline --no-latency --no-e2e"
for v in base s; do
  OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $out/fetch_$v -o pmc -- python $B > $out/bench_$v.json 2> $out/bench_$v.err || exit 99
done
