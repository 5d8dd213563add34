#!/bin/bash
# Round 5, call ZL: wave priority in br1f's rows (s_setprio; results unchanged by construction):
# var_prio1 = high priority from the row's landing barrier through the multiply-accumulate and the
# next row's DMA issue, var_prio2 = high priority through the forward transform instead; var_prio2f =
# br2f: high priority from each digit transform's cross-wave exchange to the next digit; a same-box
# A/B with var_base = HEAD, twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zl
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05zl/
