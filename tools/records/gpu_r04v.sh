# rocprofv3 kernel trace + stats of the default bench command itself (the bench line it prints
# carries the roofline whose average launch time the trace must match). OMR_COOPERATIVE=0: the
# latency leg runs br2l instead of the cooperative br2x, so the profiled process exits cleanly
# (exit-time fault).
set -o pipefail
out=gpurun_out/r04v
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OMR_COOPERATIVE=0 timeout -k 10 900 rocprofv3 --kernel-trace --stats -T -f csv -d $out/kt -o kt -- python bench.py > $out/bench.json 2> $out/bench.err || exit 1
