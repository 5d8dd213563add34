# br1f instruction-diet A/B: full GPU suite on the new build, then base vs new timing twice.
set -o pipefail
out=gpurun_out/r04f
mkdir -p $out
rm -f gpurun_out/bench_variants.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit 1
tools/bench_variants.sh 16384 --no-e2e || exit 2
tools/bench_variants.sh 16384 --no-e2e || exit 3
cp gpurun_out/bench_variants.log $out/ab.log
