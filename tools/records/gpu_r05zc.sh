#!/bin/bash
# Round 5, call ZC: the shader clock and socket power the throughput kernels run at. rocm-smi samples
# (current sclk, power) every 0.5 s in the background while bench.py runs its default D = 65,536
# steps; the sampler is stopped by its PID.
export TMPDIR=/tmp
out=gpurun_out/r05zc
mkdir -p $out
( while true; do date +%s.%N; rocm-smi -c -P -u 2>&1 | grep -E "sclk|Power|GPU use" ; sleep 0.5; done ) > $out/smi.log 2>&1 &
sp=$!
timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err
rc=$?
kill $sp
wait $sp 2>/dev/null
tail -c 600 $out/bench.json
grep -c sclk $out/smi.log
exit $rc
