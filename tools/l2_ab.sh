#!/bin/bash
# L2 behaviour of level-2 variants: TCC hit / miss pass per tfhe-omr_amd/build/var_<name>.so
#   tools/l2_ab.sh <tag> <name> [<name> ...]
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/$1; shift; mkdir -p $out
B="bench.py --steps 1 --warmup 0 --messages 16384 --no-cpu-baseline --no-latency --no-e2e"
for v in "$@"; do
  export OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T -f csv -d $out/${v}_tcc -o pmc -- python $B > $out/${v}_tcc.log 2>&1 || exit 1
  echo "done $v"
done
