#!/bin/bash
# Round 5, call C: level-2 time vs batch size for the base and the pipelined build (occupancy).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05c
for v in base pipe; do
  OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so tools/gpu_step.sh 300 r05c/occ_$v.log python -u tools/l2_occupancy.py || exit 99
done
