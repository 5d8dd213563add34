#!/bin/bash
# Single-message latency split (tools/latency_split.py) with every tfhe-omr_amd/build/var_*.so.
mkdir -p gpurun_out
for so in tfhe-omr_amd/build/var_*.so; do
  echo "== $(basename $so)" | tee -a gpurun_out/latency_variants.log
  OMR_GPU_LIB=$PWD/$so timeout -k 10 120 python tools/latency_split.py 1 7 2>&1 | tee -a gpurun_out/latency_variants.log
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
