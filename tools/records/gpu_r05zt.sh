#!/bin/bash
# Round 5, call ZT: the latency path's br2y with the bounded wave priority in its digit transforms
# (var_yp) against the HEAD (var_base): single-message latency split, three times each, alternating.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zt
for k in 1 2 3; do
  for v in base yp; do
    OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 300 python tools/latency_split.py 1 7 > gpurun_out/r05zt/ls_$v.log 2>&1 || exit 97
    echo "$v $(grep 'D=1:' gpurun_out/r05zt/ls_$v.log)" | tee -a gpurun_out/r05zt/latency_ab.log
  done
done
