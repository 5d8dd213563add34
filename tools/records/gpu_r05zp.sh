#!/bin/bash
# Round 5, call ZP: the HEAD with br2f's bounded wave priority -- the full GPU suite and smoke, then
# the default bench line ten times on one box (the slow mode of the unbounded priority, r05zn, was
# one run in four).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zp
tools/gpu_step.sh 900 r05zp/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05zp/gpu_tests.log && ! grep -q "FAILED" gpurun_out/r05zp/gpu_tests.log || { echo "suite failed"; exit 98; }
tools/gpu_step.sh 300 r05zp/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
for k in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-latency --no-e2e > gpurun_out/r05zp/b.json 2>> gpurun_out/r05zp/bench.err || exit 97
  python3 -c "import json;d=json.loads(open('gpurun_out/r05zp/b.json').readline());print($k, d['value'], d['stage_ms_per_step'])" | tee -a gpurun_out/r05zp/repeat.log
done
