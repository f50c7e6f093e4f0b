#!/bin/bash
# Round-4 measurements: the default bench line (C3 + parity_mode + CPU baseline), per-rank shard
# lines of the 8-GPU configs on one GPU (C3 256 games, C4 128 games, the C5 net at 128 boards),
# (PMC passes: tools/r4_pmc.sh)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4m
O=gpurun_out/r4m
T="timeout -k 10"
$T 600 python -u bench.py > $O/bench_c3_default.json 2> $O/bench_c3_default.err || { tail -5 $O/bench_c3_default.err; exit 1; }
tail -c 600 $O/bench_c3_default.json; echo
$T 300 python -u bench.py --global-games 256 --steps 3 --warmup 1 --cpu-baseline 0 --parity-steps 0 > $O/bench_c3_g256.json 2> $O/bench_c3_g256.err || { tail -5 $O/bench_c3_g256.err; exit 1; }
$T 300 python -u bench.py --config c4 --steps 2 --warmup 1 --cpu-baseline 0 --parity-steps 0 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
$T 300 python -u bench.py --config c4 --global-games 128 --steps 3 --warmup 1 --cpu-baseline 0 --parity-steps 0 > $O/bench_c4_g128.json 2> $O/bench_c4_g128.err || { tail -5 $O/bench_c4_g128.err; exit 1; }
for f in bench_c3_g256 bench_c4 bench_c4_g128; do python3 -c "import json,sys;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', round(d['value'],2), d['config']['games_per_gpu'], round(d['roofline']['frac'],4), d['roofline']['kernel'])"; done
for B in 1024 128; do $T 120 python -u tools/net_bench.py --game chess --batch $B --iters 10 2>&1 | tee -a $O/c5_net.txt || exit 1; done
for B in 1024 128; do $T 120 python -u tools/net_bench.py --game go19 --batch $B --iters 10 2>&1 | tee -a $O/c4_net.txt || exit 1; done
