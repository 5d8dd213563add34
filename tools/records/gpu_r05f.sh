#!/bin/bash
# Round 5, call F: the full GPU suite + smoke at the new level-2 HEAD, the default bench line, and a
# same-box A/B of the new library against the round-4 one (var_base), twice each.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05f
tools/gpu_step.sh 1000 r05f/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05f/gpu_tests.log && ! grep -q "FAILED" gpurun_out/r05f/gpu_tests.log || { echo "suite failed"; exit 98; }
tools/gpu_step.sh 300 r05f/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
tools/gpu_step.sh 600 r05f/bench.log python bench.py || exit 99
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e
cp gpurun_out/bench_variants.log gpurun_out/r05f/
