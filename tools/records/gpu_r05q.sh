#!/bin/bash
# Round 5, call Q: the HEAD after the level-2 digit-word diet and the br2y default with key-prefetch
# helpers -- the full GPU suite, smoke, then the round profile (bench line, kernel traces, PMC passes,
# RCCL rehearsal at N = 1, latency split).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05q
tools/gpu_step.sh 600 r05q/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05q/gpu_tests.log && ! grep -q "FAILED" gpurun_out/r05q/gpu_tests.log || { echo "suite failed"; exit 98; }
tools/gpu_step.sh 300 r05q/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
bash tools/profile_round.sh r05q 16384
