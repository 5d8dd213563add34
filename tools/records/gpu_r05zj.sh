#!/bin/bash
# Round 5, call ZJ: var_pka = br2f computes the next executed step's mask digit words in the current
# step's tail (after the barrier that follows every thread's mask update, beside the last inverses)
# instead of after the step-start barrier; parity and timed-geometry tests through it, then a
# same-box A/B with var_base = HEAD, twice.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05zj
OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_pka.so tools/gpu_step.sh 700 r05zj/tests_pka.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_timed_geometry.py -v --timeout 300 --timeout-method thread || exit 99
grep -q "passed" gpurun_out/r05zj/tests_pka.log && ! grep -q "FAILED" gpurun_out/r05zj/tests_pka.log || { echo "tests failed"; exit 98; }
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 65536 --no-e2e && tools/bench_variants.sh 65536 --no-e2e || exit 97
cp gpurun_out/bench_variants.log gpurun_out/r05zj/
