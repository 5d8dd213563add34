#!/bin/bash
# Round 5, call ZO: a bounded wave priority in br2f (var_pb: s_setprio 2 only from each digit
# transform's cross-wave barrier to the end of its multiply-accumulates, 0 otherwise) against the
# HEAD (var_base, no priority), alternating, eight times each on one box: does the bimodal slow mode
# of r05zn (unbounded priority) stay away?
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zo
rm -f gpurun_out/bench_variants.log
for k in 1 2 3 4 5 6 7 8; do tools/bench_variants.sh 65536 --no-e2e || exit 97; done
cp gpurun_out/bench_variants.log gpurun_out/r05zo/
