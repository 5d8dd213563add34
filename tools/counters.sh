#!/bin/bash
# SQ counter passes for the detect kernels (one rocprofv3 --pmc pass per group, kernel-trace off).
# usage: tools/counters.sh <tag> <D> "<group1>" "<group2>" ...
tag=$1; D=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 60 rocprofv3 -L > $out/counters_list.txt 2>&1
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -T -f csv -d $out/pmc$i -o pmc -- python bench.py --steps 1 --warmup 0 --messages $D --no-cpu-baseline --no-latency > $out/pmc$i.log 2>&1
  rc=$?
  echo "[counters] group $i ($grp) rc=$rc" | tee -a $out/steps.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
