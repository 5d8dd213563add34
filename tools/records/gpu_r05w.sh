#!/bin/bash
# Round 5, call W: the co-scheduled pipeline (dual_kernel: level 1 of chunk k + 1 beside level 2 of
# chunk k) -- its parity test against the sequential launches, then bench.py at D = 65,536 with
# OMR_DUAL=1 (4 and 8 chunks) against the default, twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05w
tools/gpu_step.sh 400 r05w/dual_parity.log python -u -m pytest tests/test_gpu_timed_geometry.py -m gpu -v --timeout 300 --timeout-method thread -k dual || exit 99
grep -q "passed" gpurun_out/r05w/dual_parity.log && ! grep -q "FAILED" gpurun_out/r05w/dual_parity.log || { echo "parity failed"; exit 98; }
B="bench.py --messages 65536 --steps 1 --warmup 1 --no-cpu-baseline --no-latency --no-e2e"
for rep in 1 2; do
  tools/gpu_step.sh 300 r05w/bench_seq_$rep.json python $B || exit 99
  OMR_DUAL=1 OMR_DUAL_CHUNKS=4 tools/gpu_step.sh 300 r05w/bench_dual4_$rep.json python $B || exit 99
  OMR_DUAL=1 OMR_DUAL_CHUNKS=8 tools/gpu_step.sh 300 r05w/bench_dual8_$rep.json python $B || exit 99
done
for f in gpurun_out/r05w/bench_*.json; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["correct"])')"; done
