# configs[3] (D = 524,288 total, strong scaling) and configs[4] (D = 2^20: detect + encode +
# retrieval) at N = 1 on the round-4 HEAD.
set -o pipefail
out=gpurun_out/r04t
mkdir -p $out
timeout -k 10 500 python bench.py --total-messages 524288 --steps 1 --warmup 1 --no-cpu-baseline > $out/bench_strong_d524288_n1.json 2> $out/strong.err || exit 1
timeout -k 10 700 python bench.py --total-messages 1048576 --steps 1 --warmup 0 --no-cpu-baseline > $out/bench_d2p20_n1.json 2> $out/d2p20.err || exit 2
