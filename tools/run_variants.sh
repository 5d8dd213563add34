#!/bin/bash
# Time every tfhe-omr_amd/build/var_*.so with tools/quick_perf.py (stops on a crash/timeout).
D=${1:-4096}
mkdir -p gpurun_out
for so in tfhe-omr_amd/build/var_*.so; do
  OMR_GPU_LIB=$PWD/$so timeout -k 10 300 python tools/quick_perf.py $D 2 >> gpurun_out/variants.log 2>&1
  rc=$?
  echo "[variants] $so rc=$rc" >> gpurun_out/variants.log
  case $rc in 0) ;; *) tail -5 gpurun_out/variants.log; exit $rc;; esac
done
cat gpurun_out/variants.log
