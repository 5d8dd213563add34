#!/bin/bash
# Same-box sweep of the detect chunk size (omr_ctx_set_batch) at D messages; stops on a crash/timeout.
#   tools/batch_sweep.sh [D] [batch ...]
D=${1:-65536}; shift
mkdir -p gpurun_out
[ $# -gt 0 ] || set -- 16384 32768 65536 16384
for B in "$@"; do
  timeout -k 10 300 python bench.py --messages $D --batch $B --steps 2 --warmup 1 --no-cpu-baseline --no-latency > gpurun_out/bs.json 2>> gpurun_out/batch_sweep.err
  rc=$?
  echo "batch=$B rc=$rc $(python3 -c "import json;d=json.loads(open('gpurun_out/bs.json').readline());print(d['value'],d['ms_per_step'],d['stage_ms_per_step'],d['correct'],d['e2e']['ok'] if d['e2e'] else None)" 2>&1)" | tee -a gpurun_out/batch_sweep.log
  case $rc in 0) ;; *) exit $rc;; esac
done
