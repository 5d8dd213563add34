# br1f ablation 2: buffer DMA + peeled first row (lambda form), with each of floor rounding, H/2 offset, v_and_or addresses; twice.
# (Record of a round-4 A/B: the var_*.so it times were built by tools/build_variant.sh from scratch
# edits / -D switches that were folded into or removed from the sources afterwards)
set -o pipefail
out=gpurun_out/r04h
mkdir -p $out
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 16384 --no-e2e || exit 2
tools/bench_variants.sh 16384 --no-e2e || exit 3
cp gpurun_out/bench_variants.log $out/ab.log
