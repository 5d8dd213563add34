# Round-4 HEAD validation: full GPU suite, smoke, a 5-step bench.
set -o pipefail
out=gpurun_out/r04e
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > $out/bench.json 2> $out/bench.err || exit 3
