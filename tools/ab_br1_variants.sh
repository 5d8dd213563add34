#!/bin/bash
# Same-box A/B of library variants (round 6): parity tests through each non-base variant, then bench.py
# at D = 65,536 (2 timed steps) for every variant, alternating, twice.
#   tools/ab_br1_variants.sh <tag> <variant>...     (tfhe-omr_amd/build/var_<variant>.so)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  [ "$v" = base ] && continue
  OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/parity_$v.log 2>&1 || { tail -30 $out/parity_$v.log; exit 97; }
  echo "parity $v: $(tail -1 $out/parity_$v.log)" | tee -a $out/ab.log
done
for k in 1 2; do
  for v in "$@"; do
    OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 300 python bench.py --messages 65536 --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-e2e > $out/bv_$v.json 2>> $out/bv.err || exit 98
    echo "$v $(python3 -c "import json;d=json.loads(open('$out/bv_$v.json').readline());print(d['value'],'L1',d['per_step_spread']['level1_rotation_ms']['median'],'L2',d['per_step_spread']['level2_rotation_ms']['median'],d['correct'],d['exactness']['guarded_output_identical'])")" | tee -a $out/ab.log
  done
done
