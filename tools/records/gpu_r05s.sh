#!/bin/bash
# Round 5, call S: phase trace of the latency path with br2y_kernel (the default) and its helpers.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05s
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/aux/phase.so tools/gpu_step.sh 300 r05s/phase_br2y.log python tools/phase_trace.py || exit 99
