#!/bin/bash
# Round 5, call X: why the co-scheduled pipeline is no faster -- instruction-cache and VALU counters
# of one 16,384-message detect with OMR_DUAL=1 (4 chunks) and without.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05x
B="bench.py --steps 1 --warmup 0 --messages 16384 --no-cpu-baseline --no-latency --no-e2e"
for mode in seq dual; do
  if [ $mode = dual ]; then export OMR_DUAL=1 OMR_DUAL_CHUNKS=4; fi
  timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU -T -f csv -d gpurun_out/r05x/pmc_$mode -o pmc -- python $B > gpurun_out/r05x/$mode.log 2>&1 || { echo "pmc $mode failed"; exit 99; }
done
