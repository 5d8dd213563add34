#!/bin/bash
# Round profile on the GPU box (one call): default bench line, rocprofv3 kernel trace + stats of
# one 16,384-message detect step and of single-message latency calls, separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, two SQ groups), and the RCCL rehearsal of the multi-GPU path at N = 1.
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
run 300 python bench.py --messages 4096 --steps 1 --warmup 1 --force-dist --no-cpu-baseline > $out/bench_forcedist_rccl_n1.json 2> $out/forcedist.err
tail -1 $out/bench_forcedist_rccl_n1.json
# last: a process that made cooperative launches (the latency path's two-CU / five-CU kernels)
# faults at exit under rocprofv3: libamdhip64's exit handler -> libhsa-runtime64 teardown, after the
# profiler tool has finalised (its trace and stats are complete). Not this library's code: the same
# workload without cooperative launches (OMR_COOPERATIVE=0 or threshold 0) exits 0, with torch's
# bundled HIP runtime it faults the same way, and hipDeviceReset before exit does not avoid it
# (profiles/r04/exit_fault_*). So nothing runs after it.
run 300 rocprofv3 --kernel-trace --stats -T -f csv -d $out/kt_latency -o kt -- python tools/latency_split.py 1 7
find $out -name "*.csv" | head -30
