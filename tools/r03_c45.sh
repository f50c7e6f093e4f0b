#!/bin/bash
# Round 3: the C4 (Go 19x19, 1024 games, 800 sims) bench line with its parity_mode on the final tree,
# and the C5 network shape (chess 8x8x111 -> 4672, 1024 boards) forward in both trunk precisions.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03l_c45
mkdir -p $O
timeout -k 10 600 python3 bench.py --config c4 --cpu-baseline 0 --steps 2 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { echo C4_FAIL; tail -20 $O/bench_c4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c4.json'));print('c4', round(d['value'],2), 'pos/s', d['roofline']['kernel'], round(d['roofline']['frac'],4), 'parity', d.get('parity_mode',{}).get('value'))"
for p in fp16 bf16x3; do
  timeout -k 10 120 python3 tools/net_bench.py --game chess --batch 1024 --precision $p --iters 10 > $O/c5_$p.txt 2>&1 || { echo C5_FAIL $p; tail -5 $O/c5_$p.txt; exit 1; }
  tail -1 $O/c5_$p.txt
done
