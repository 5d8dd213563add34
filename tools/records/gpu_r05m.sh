#!/bin/bash
# Round 5, call M: why br2y_kernel is slower than br2x -- the latency split with the key loads
# skipped (timing-only ablation var_nokey, wrong output), against var_y and br2x (OMR_BR2Y=0).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05m
for v in y nokey; do
  OMR_BR2Y=1 OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so tools/gpu_step.sh 300 r05m/latency_$v.log python tools/latency_split.py 1 7 || exit 99
done
OMR_BR2Y=0 OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_y.so tools/gpu_step.sh 300 r05m/latency_br2x.log python tools/latency_split.py 1 7 || exit 99
