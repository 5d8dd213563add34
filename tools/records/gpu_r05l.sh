#!/bin/bash
# Round 5, call L: the two-CU FFT latency kernel (br2y_kernel) -- its parity tests first (against
# the exact NTT two-CU kernel and the oracle), then the latency split with br2y and with br2x
# (OMR_BR2Y=0), then the default bench line.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05l
tools/gpu_step.sh 600 r05l/gpu_parity.log python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05l/gpu_parity.log && ! grep -q "FAILED" gpurun_out/r05l/gpu_parity.log || { echo "parity failed"; exit 98; }
tools/gpu_step.sh 300 r05l/latency_br2y.log python tools/latency_split.py 1 7 64 || exit 99
OMR_BR2Y=0 tools/gpu_step.sh 300 r05l/latency_br2x.log python tools/latency_split.py 1 7 64 || exit 99
tools/gpu_step.sh 300 r05l/latency_br2y_2.log python tools/latency_split.py 1 7 64 || exit 99
tools/gpu_step.sh 600 r05l/bench.log python bench.py || exit 99
