#!/bin/bash
# On the GPU box: bench line + rocprofv3 kernel-trace/stats + separate PMC passes (FETCH_SIZE,
# WRITE_SIZE) for the detect pipeline. Outputs under gpurun_out/<tag>/. Each GPU step has its own
# time limit; the script stops at the first crash/timeout.
set -o pipefail
tag=${1:-r01}
D=${2:-16384}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { local secs=$1; shift; timeout -k 10 "$secs" "$@"; local rc=$?; echo "[profile] rc=$rc: $*" >> $out/steps.log;
        if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 600 python bench.py > $out/bench.json 2> $out/bench.err
tail -1 $out/bench.json
run 300 rocprofv3 --kernel-trace --stats -T -f csv -d $out/kt -o kt -- python bench.py --steps 1 --warmup 0 --messages $D --no-cpu-baseline --no-latency
run 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $out/pmc_fetch -o pmc -- python bench.py --steps 1 --warmup 0 --messages $D --no-cpu-baseline --no-latency
run 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $out/pmc_write -o pmc -- python bench.py --steps 1 --warmup 0 --messages $D --no-cpu-baseline --no-latency
find $out -name "*.csv" | head -20
