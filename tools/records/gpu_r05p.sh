#!/bin/bash
# Round 5, call P: br2y_kernel with L2 key-prefetch helper workgroups -- its parity test against
# br2x, then the latency split (br2x default; br2y with and without helpers), twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05p
tools/gpu_step.sh 300 r05p/parity.log python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "fft_two_cu or latency" || exit 99
grep -q "passed" gpurun_out/r05p/parity.log && ! grep -q "FAILED" gpurun_out/r05p/parity.log || { echo "parity failed"; exit 98; }
for rep in 1 2; do
  tools/gpu_step.sh 300 r05p/latency_br2x_$rep.log python tools/latency_split.py 1 7 || exit 99
  OMR_BR2Y=1 tools/gpu_step.sh 300 r05p/latency_br2y_pf_$rep.log python tools/latency_split.py 1 7 || exit 99
  OMR_BR2Y=1 OMR_PREFETCH=0 tools/gpu_step.sh 300 r05p/latency_br2y_nopf_$rep.log python tools/latency_split.py 1 7 || exit 99
done
