#!/bin/bash
# Round 5, final call: the HEAD with br2f's bounded wave priority in the digit transforms and the
# inverses -- the full GPU suite, smoke, the default bench line, six more timing-only bench runs
# (run-to-run spread), then the round profile (kernel traces, counters, latency split).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zr
tools/gpu_step.sh 900 r05zr/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05zr/gpu_tests.log && ! grep -q "FAILED" gpurun_out/r05zr/gpu_tests.log || { echo "suite failed"; exit 98; }
tools/gpu_step.sh 300 r05zr/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
for k in 1 2 3 4 5 6; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-latency --no-e2e > gpurun_out/r05zr/b.json 2>> gpurun_out/r05zr/repeat.err || exit 97
  python3 -c "import json;d=json.loads(open('gpurun_out/r05zr/b.json').readline());print($k, d['value'], d['stage_ms_per_step'])" | tee -a gpurun_out/r05zr/repeat.log
done
bash tools/profile_round.sh r05zr 16384
