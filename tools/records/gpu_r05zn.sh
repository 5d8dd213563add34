#!/bin/bash
# Round 5, call ZN: run-to-run spread of br2f with and without the wave priority (var_base = HEAD
# with s_setprio, var_noprio = the library before it), alternating, four times each on one box:
# r05zm saw two single runs of the priority kernel 45 % and 60 % slower at level 2.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zn
rm -f gpurun_out/bench_variants.log
for k in 1 2 3 4; do tools/bench_variants.sh 65536 --no-e2e || exit 97; done
cp gpurun_out/bench_variants.log gpurun_out/r05zn/
