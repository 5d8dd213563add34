#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a crash/timeout.
# usage: tools/gpu_step.sh <seconds> <logfile> <cmd...>   (pytest failures rc=1 are not fatal)
secs=$1; log=$2; shift 2
mkdir -p "$(dirname "gpurun_out/$log")"
timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "[gpu_step] $* -> rc=$rc" | tee -a gpurun_out/steps.log
tail -40 "gpurun_out/$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 99; fi
exit 0
