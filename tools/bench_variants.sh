#!/bin/bash
# bench.py (one timed step at D messages) with every tfhe-omr_amd/build/var_*.so; stops on a crash/timeout.
#   tools/bench_variants.sh [D] [extra bench.py flags, e.g. --no-e2e for timing-only ablation builds]
D=${1:-65536}
shift
mkdir -p gpurun_out
for so in tfhe-omr_amd/build/var_*.so; do
  OMR_GPU_LIB=$PWD/$so timeout -k 10 300 python bench.py --messages $D --steps 1 --warmup 1 --no-cpu-baseline --no-latency "$@" > gpurun_out/bv.json 2>> gpurun_out/bench_variants.err
  rc=$?
  echo "$(basename $so) rc=$rc $(python3 -c "import json;d=json.loads(open('gpurun_out/bv.json').readline());print(d['value'],d['ms_per_step'],d['stage_ms_per_step'],d['correct'],d['e2e']['ok'] if d['e2e'] else None)" 2>&1)" | tee -a gpurun_out/bench_variants.log
  case $rc in 0) ;; *) exit $rc;; esac
done
