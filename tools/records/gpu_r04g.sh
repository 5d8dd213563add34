# br1f instruction-diet ablation: base (HEAD), all changes, without the buffer DMA, without the
# peeled first row, representation only (+ SGPR wave), representation only (VGPR wave); twice.
# (Record of a round-4 A/B: the var_*.so it times were built by tools/build_variant.sh from scratch
# edits / -D switches that were folded into or removed from the sources afterwards)
set -o pipefail
out=gpurun_out/r04g
mkdir -p $out
rm -f gpurun_out/bench_variants.log
tools/bench_variants.sh 16384 --no-e2e || exit 2
tools/bench_variants.sh 16384 --no-e2e || exit 3
cp gpurun_out/bench_variants.log $out/ab.log
