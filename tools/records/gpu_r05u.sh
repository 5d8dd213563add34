#!/bin/bash
# Round 5, call U: br2y's same-XCD hand-off (plain stores into the XCD's L2 when both workers share
# one) -- the latency parity tests, then the latency split (HEAD; OMR_FAST_HANDOFF=0; the no-hand-off
# timing ablation) twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05u
tools/gpu_step.sh 300 r05u/parity.log python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "fft_two_cu or latency" || exit 99
grep -q "passed" gpurun_out/r05u/parity.log && ! grep -q "FAILED" gpurun_out/r05u/parity.log || { echo "parity failed"; exit 98; }
for rep in 1 2; do
  tools/gpu_step.sh 300 r05u/latency_head_$rep.log python tools/latency_split.py 1 7 || exit 99
  OMR_FAST_HANDOFF=0 tools/gpu_step.sh 300 r05u/latency_sc1_$rep.log python tools/latency_split.py 1 7 || exit 99
  OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/aux/noho.so tools/gpu_step.sh 300 r05u/latency_noho_$rep.log python tools/latency_split.py 1 7 || exit 99
done
