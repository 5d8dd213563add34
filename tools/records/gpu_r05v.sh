#!/bin/bash
# Round 5, call V: occupancy experiment -- both blind rotations with their LDS padded to 82 KB so one
# workgroup fits per CU (var_pad1, -DOMR_BR1_PAD1 -DOMR_BR2_PAD1) against the library (var_base):
# how much of each level's throughput one workgroup per CU keeps (for a level-1 / level-2
# co-scheduled design).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05v
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05v/
