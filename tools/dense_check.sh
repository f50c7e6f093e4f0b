#!/bin/bash
# DENSE v6 geometry (conv flag 8) vs the padded geometry: A/B timing per board, and the conv1 split skip.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/dense
mkdir -p $O
for g in gomoku15 go19 chess go13 gomoku9; do
  timeout -k 10 200 python3 tools/net_bench.py --game $g --batch 2048 --flags 0x4,0xc --iters 5 --rounds 3 > $O/nb_$g.txt 2>&1 || { echo NB_FAIL $g; tail -5 $O/nb_$g.txt; exit 1; }
  echo $g; cat $O/nb_$g.txt
done
timeout -k 10 200 python3 tools/net_bench.py --game go19 --batch 1024 --flags 0x4,0xc --iters 5 --rounds 3 > $O/nb_go19_1024.txt 2>&1 && { echo go19 B=1024; cat $O/nb_go19_1024.txt; }
