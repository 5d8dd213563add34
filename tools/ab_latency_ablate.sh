#!/bin/bash
# Timing-only ablations of the latency path's level 2 (round 6): tools/latency_split.py (1 and 7
# messages) through the base library and the br2y ablation builds (wrong output: no parity run),
# alternating, twice.
#   tools/ab_latency_ablate.sh <tag> <variant>...     (tfhe-omr_amd/build/var_<variant>.so)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for k in 1 2; do
  for v in "$@"; do
    OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 200 python tools/latency_split.py 1 7 > $out/ls_$v.log 2>&1 || exit 98
    echo "$v $(grep 'D=1:' $out/ls_$v.log) | $(grep 'D=7:' $out/ls_$v.log)" | tee -a $out/ab.log
  done
done
