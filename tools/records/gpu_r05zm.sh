#!/bin/bash
# Round 5, call ZM: br2f wave-priority follow-ups (results unchanged by construction): var_pinv =
# the inverses too (0 at each inverse's start, 2 after its cross-wave barrier), var_p3 = priority 3
# instead of 2 after the forward's barrier, var_ptr = the FFT trace's digit transforms the same way;
# a same-box A/B with var_base = HEAD, twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zm
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05zm/
