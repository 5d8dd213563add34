#!/bin/bash
# Round 5, call ZS: br1f wave priority in its barrier-free phases -- var_b1inv: raised through the
# step's inverse pair and accumulator update; var_b1dig: raised through the step's digit words;
# against var_base = HEAD, three times each, alternating.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zs
rm -f gpurun_out/bench_variants.log
for k in 1 2 3; do tools/bench_variants.sh 65536 --no-e2e || exit 97; done
cp gpurun_out/bench_variants.log gpurun_out/r05zs/
