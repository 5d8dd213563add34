#!/bin/bash
# Round profile on the GPU box (one call): default bench line, rocprofv3 kernel trace + stats of
# one 16,384-message detect step and of single-message latency calls, separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, two SQ groups, the L1 -> L2 read requests and L2 hits / misses), and the RCCL rehearsal of the multi-GPU path at N = 1.
# Every GPU step has its own time limit; the script stops at the first failure.
# usage: tools/profile_round.sh <tag> [D]
set -o pipefail
tag=${1:-r02}
D=${2:-16384}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; echo "[profile] rc=$rc: $*" >> $out/steps.log;
        if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
B="bench.py --steps 1 --warmup 0 --messages $D --no-cpu-baseline --no-latency --no-e2e"
run 600 python bench.py > $out/bench.json 2> $out/bench.err
tail -1 $out/bench.json
run 300 rocprofv3 --kernel-trace --stats -T -f csv -d $out/kt -o kt -- python $B
run 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $out/pmc_fetch -o pmc -- python $B
run 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $out/pmc_write -o pmc -- python $B
run 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 -T -f csv -d $out/pmc1 -o pmc -- python $B
run 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_LDS -T -f csv -d $out/pmc2 -o pmc -- python $B
run 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -T -f csv -d $out/pmc_l2 -o pmc -- python $B
run 300 python bench.py --messages 4096 --steps 1 --warmup 1 --force-dist --no-cpu-baseline > $out/bench_forcedist_rccl_n1.json 2> $out/forcedist.err
tail -1 $out/bench_forcedist_rccl_n1.json
# The single-message latency split as it runs (cooperative two-CU / five-CU kernels), unprofiled,
# then its kernel trace with OMR_COOPERATIVE=0 (br2l / trace_kernel instead of br2x / trace_x): a
# profiled process that made a cooperative launch faults in the HIP/HSA runtime's exit-time teardown
# after the tool has finalised (tools/coop_min.hip reproduces it with no library state,
# profiles/r05/coop_min_exit_fault.md), so the profiled step avoids them and the round exits 0.
run 300 python tools/latency_split.py 1 7 > $out/latency_split.log
OMR_COOPERATIVE=0 run 300 rocprofv3 --kernel-trace --stats -T -f csv -d $out/kt_latency -o kt -- python tools/latency_split.py 1 7
find $out -name "*.csv" | head -30
