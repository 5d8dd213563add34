#!/bin/bash
# Round 5, call Z: the round profile at the HEAD with the FFT trace -- smoke, bench line, kernel
# traces, SQ / FETCH / WRITE / L1->L2 passes, RCCL rehearsal at N = 1, latency split.
export TMPDIR=/tmp
mkdir -p gpurun_out/r05z
tools/gpu_step.sh 300 r05z/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 99
bash tools/profile_round.sh r05z 16384
