#!/bin/bash
# Round 5, call ZQ: the bounded wave priority extended -- var_pib: br2f's inverses raised from their
# cross-wave barrier to their end; var_ptb: the FFT trace's digits as br2f's (raised from the
# transform's cross-wave barrier to the end of the products); against var_base = HEAD, five times
# each, alternating, on one box.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zq
rm -f gpurun_out/bench_variants.log
for k in 1 2 3 4 5; do tools/bench_variants.sh 65536 --no-e2e || exit 97; done
cp gpurun_out/bench_variants.log gpurun_out/r05zq/
