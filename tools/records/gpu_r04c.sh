# Exit-time fault probes under rocprofv3 (least likely to fault first; a fault ends the call).
set -o pipefail
out=gpurun_out/r04c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
prof() { local tag=$1; shift; timeout -k 10 150 rocprofv3 --kernel-trace --stats -T -f csv -d $out/kt_$tag -o kt -- python tools/exit_fault_probe.py "$@" > $out/probe_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc" >> $out/probes.log; return $rc; }
prof thr thr && OMR_COOPERATIVE=0 prof nocoop coop && prof torch torch && prof reset reset && prof coop coop
