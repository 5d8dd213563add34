#!/bin/bash
# Same-box A/B of the latency path's level 2: br2y (default) vs br2z (OMR_BR2Z=1, four CUs per
# message). The four-CU parity test first, then tools/latency_split.py (1 and 7 messages) for both,
# alternating, twice.
#   tools/ab_br2z.sh <tag>
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "four_cu or two_cu" --timeout 240 --timeout-method thread > $out/parity.log 2>&1 || { tail -40 $out/parity.log; exit 97; }
echo "parity: $(tail -1 $out/parity.log)" | tee -a $out/ab.log
for k in 1 2; do
  for z in 0 1; do
    OMR_BR2Z=$z timeout -k 10 200 python tools/latency_split.py 1 7 > $out/ls_z$z.log 2>&1 || exit 98
    echo "br2z=$z $(grep 'D=1:' $out/ls_z$z.log) | $(grep 'D=7:' $out/ls_z$z.log)" | tee -a $out/ab.log
  done
done
