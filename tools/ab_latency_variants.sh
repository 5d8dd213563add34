#!/bin/bash
# Same-box A/B of library variants on the latency path (round 6): the br2y parity test through each
# non-base variant, then tools/latency_split.py (1 and 7 messages) for every variant, alternating, twice.
#   tools/ab_latency_variants.sh <tag> <variant>...     (tfhe-omr_amd/build/var_<variant>.so)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  [ "$v" = base ] && continue
  OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "latency" --timeout 240 --timeout-method thread > $out/parity_$v.log 2>&1 || { tail -30 $out/parity_$v.log; exit 97; }
  echo "parity $v: $(tail -1 $out/parity_$v.log)" | tee -a $out/ab.log
done
for k in 1 2; do
  for v in "$@"; do
    OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 200 python tools/latency_split.py 1 7 > $out/ls_$v.log 2>&1 || exit 98
    echo "$v $(grep 'D=1:' $out/ls_$v.log) | $(grep 'D=7:' $out/ls_$v.log)" | tee -a $out/ab.log
  done
done
