#!/bin/bash
# On the GPU box: the -m gpu parity suite, then one default bench line. Each GPU step has its own
# time limit; the script stops at the first crash / timeout (tools/gpu_step.sh).
set -o pipefail
tag=${1:-check}
mkdir -p gpurun_out/$tag
tools/gpu_step.sh 600 $tag/gpu_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread &&
tools/gpu_step.sh 400 $tag/bench.log python bench.py
