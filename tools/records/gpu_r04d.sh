# Exit-time fault: the reset probe, then the same rocprofv3 command as round 3's failing step.
set -o pipefail
out=gpurun_out/r04d
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
prof() { local tag=$1; shift; timeout -k 10 150 rocprofv3 --kernel-trace --stats -T -f csv -d $out/kt_$tag -o kt -- python "$@" > $out/prof_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc" >> $out/probes.log; return $rc; }
prof reset tools/exit_fault_probe.py reset && prof latency_split tools/latency_split.py 1 7 && OMR_KEEP_DEVICE=1 prof latency_split_keep tools/latency_split.py 1 7
