#!/bin/bash
# Round 5, final call: the full GPU suite, smoke, then the round profile at the HEAD (bench line,
# kernel traces, SQ / FETCH / WRITE / L1->L2 passes, RCCL rehearsal at N = 1, latency split).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zz
tools/gpu_step.sh 900 r05zz/gpu_tests.log python -u -m pytest tests -m gpu -v -rP --timeout 600 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05zz/gpu_tests.log && ! grep -q "FAILED" gpurun_out/r05zz/gpu_tests.log || { echo "suite failed"; exit 98; }
tools/gpu_step.sh 300 r05zz/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
bash tools/profile_round.sh r05zz 16384
