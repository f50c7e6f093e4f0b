#!/bin/bash
# Board power and clocks while the C3 trunk runs (tools/net_bench.py, B = 2048, v7) and while idle:
# is the trunk conv power-limited?  Read-only rocm-smi / amd-smi queries (no setting is changed).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-power}
mkdir -p $O
( timeout -k 10 120 rocm-smi --showpower --showclocks --showmaxpower 2>&1 || true ) > $O/idle.txt
timeout -k 10 200 python3 tools/net_bench.py --batch 2048 --iters 2500 > $O/nb.txt 2>&1 &
NB=$!
sleep 15
for i in 1 2 3 4 5 6; do ( timeout -k 5 30 rocm-smi --showpower --showclocks 2>&1 || true ) >> $O/busy.txt; sleep 2; done
wait $NB
tail -1 $O/nb.txt
echo "== idle"; grep -iE "power|sclk|mclk|fclk" $O/idle.txt | head -12
echo "== busy"; grep -iE "power|sclk" $O/busy.txt | head -20
