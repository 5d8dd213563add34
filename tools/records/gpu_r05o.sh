#!/bin/bash
# Round 5, call O: where the latency path's time goes -- phase trace of br1l / br2x (clock64 marks,
# -DOMR_PHASE_TRACE build), the latency split on br2x (default) and br2y (OMR_BR2Y=1), and br2y with
# its key loads skipped after the first step (timing-only ablation -DOMR_BR2Y_NOKEY, wrong output).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05o
A=$PWD/tfhe-omr_amd/build/aux
OMR_GPU_LIB=$A/phase.so tools/gpu_step.sh 300 r05o/phase.log python tools/phase_trace.py || exit 99
tools/gpu_step.sh 300 r05o/latency_br2x.log python tools/latency_split.py 1 7 || exit 99
OMR_BR2Y=1 tools/gpu_step.sh 300 r05o/latency_br2y.log python tools/latency_split.py 1 7 || exit 99
OMR_BR2Y=1 OMR_GPU_LIB=$A/nokey.so tools/gpu_step.sh 300 r05o/latency_br2y_nokey.log python tools/latency_split.py 1 7 || exit 99
tools/gpu_step.sh 120 r05o/microbench_l2.log tools/microbench_l2 || exit 99
