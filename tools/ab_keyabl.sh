#!/bin/bash
# Timing-only ablation of the level-2 key stream (round 6): bench.py at D = 65,536 through the base
# library and var_keyabl (tools/build_variant.sh keyabl -DOMR_BR2_KEYABL: every key load from one 4 KB
# block, wrong output), alternating, twice.
set -o pipefail
out=gpurun_out/r06o; mkdir -p $out
for k in 1 2; do for v in base keyabl; do
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 300 python bench.py --messages 65536 --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-e2e > $out/bv_$v.json 2>> $out/bv.err || exit 98
echo "$v $(python3 -c "import json;d=json.loads(open('$out/bv_$v.json').readline());print(d['value'],'L1',d['per_step_spread']['level1_rotation_ms']['median'],'L2',d['per_step_spread']['level2_rotation_ms']['median'],d['correct'])")" | tee -a $out/ab.log
done; done
