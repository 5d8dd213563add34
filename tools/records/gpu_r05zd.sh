#!/bin/bash
# Round 5, call ZD: br2f's next-step key prefetch (the body's last digit loads the next step's first
# row instead of reloading its own) -- parity of the level-2 throughput family, then a same-box A/B
# (var_base = HEAD, var_kpf = the prefetch, var_kpi = the prefetch + the four inverses pipelined in barrier stages) twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zd
tools/gpu_step.sh 600 r05zd/tests.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_timed_geometry.py -v --timeout 300 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05zd/tests.log && ! grep -q "FAILED" gpurun_out/r05zd/tests.log || { echo "tests failed"; exit 98; }
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05zd/
