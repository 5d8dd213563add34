#!/bin/bash
# Build a variant of libomr_gpu.so with extra -D flags into tfhe-omr_amd/build/var_<name>.so
# (run on the CPU here; tools/bench_variants.sh times every var_*.so on the GPU box).
#   tools/build_variant.sh <name> [-DMACRO=VALUE ...]
set -e
name=$1; shift
cd "$(dirname "$0")/../tfhe-omr_amd"
out=build/var_$name
mkdir -p $out
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wall -Wno-unused-result -Wno-unused-function -I../include"
pids=()
for s in keygen keygen_gpu context retriever; do
  /opt/rocm/bin/hipcc $FLAGS "$@" -c csrc/$s.hip -o $out/$s.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out.so $out/*.o -lpthread
echo "built $out.so ($*)"
