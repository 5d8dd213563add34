#!/bin/bash
# Build experiment variants of libomr_gpu as build/var_<name>.so (same sources, different -D).
set -e
mk() { name=$1; shift
  mkdir -p build/var_$name
  for s in keygen keygen_gpu context retriever; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -I../include "$@" -c csrc/$s.hip -o build/var_$name/$s.o &
  done; wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/var_$name.so build/var_$name/*.o -lpthread
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -I../include "$@" --cuda-device-only -S csrc/context.hip -o /dev/null -Rpass-analysis=kernel-resource-usage 2> build/var_$name/ru.txt
  echo "== $name $*"; python3 ../tools/resource_usage.py build/var_$name/ru.txt | grep -E "br1|br2"
}
for v in "$@"; do eval "mk $v"; done
