# Validation after the level-2 and latency-kernel instruction diet (br2f buffer-descriptor key loads
# and signed digit fields; br1l offset accumulator and LDS pass-0 twiddles; br2x / br2l LDS pass-0
# twiddles): full GPU suite, smoke, a 5-step bench, then single-message latency base vs b4.
set -o pipefail
out=gpurun_out/r04l
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > $out/bench.json 2> $out/bench.err || exit 3
for v in base b4 base b4; do OMR_KEEP_DEVICE=1 OMR_GPU_LIB=$PWD/tfhe-omr_amd/build/var_$v.so timeout -k 10 120 python tools/latency_split.py 1 7 > $out/lat_$v.log 2>&1 && echo "$v $(cat $out/lat_$v.log | tr '\n' ' ')" >> $out/lat_ab.log || exit 5; done
