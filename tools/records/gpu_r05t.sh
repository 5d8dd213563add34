#!/bin/bash
# Round 5, call T: what the two-CU hand-off costs br2y -- latency split with the hand-off's payload
# stores, partner poll and payload loads removed (timing-only ablation -DOMR_BR2Y_NOHANDOFF, wrong
# output) against the library, twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05t
for rep in 1 2; do
  tools/gpu_step.sh 300 r05t/latency_head_$rep.log python tools/latency_split.py 1 7 || exit 99
  OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/aux/noho.so tools/gpu_step.sh 300 r05t/latency_noho_$rep.log python tools/latency_split.py 1 7 || exit 99
done
