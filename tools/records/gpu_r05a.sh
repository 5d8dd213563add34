#!/bin/bash
# Round 5, call A: the GPU suite after the exactness contract / bench rehearsal changes, then the
# cooperative-launch exit-fault probe (control first; the cooperative one last: it may exit 139).
export TMPDIR=/tmp
mkdir -p gpurun_out/r05a
tools/gpu_step.sh 1000 r05a/gpu_tests.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 99
tools/gpu_step.sh 120 r05a/coop_plain.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05a/coop_plain -o kt -- ./tools/coop_min plain || exit 99
tools/gpu_step.sh 120 r05a/coop_coop.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05a/coop_coop -o kt -- ./tools/coop_min coop
