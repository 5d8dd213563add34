#!/bin/bash
# Round 5, call ZK (final): the full GPU suite, smoke and the default bench line at the round-5 HEAD.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zk
tools/gpu_step.sh 900 r05zk/gpu_tests.log python -u -m pytest tests -m gpu -v -rP --timeout 600 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05zk/gpu_tests.log && ! grep -q "FAILED" gpurun_out/r05zk/gpu_tests.log || { echo "suite failed"; exit 98; }
tools/gpu_step.sh 300 r05zk/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
tools/gpu_step.sh 600 r05zk/bench.json python bench.py || exit 99
