#!/bin/bash
# conv3x3_v9x3 first-round stagger sweep (f16x3, C3 B = 2048 and C4 B = 1024), and the C2 bench's
# per-kernel times with the block-per-board FC finish / 8-slice x3 FC heads
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/stag
mkdir -p $O
L=$PWD/alphazero-multi-game_amd/build_dev/libaz_hip.so
for r in 1 2; do
  for sg in 0 8000 16000 32000 64000; do
    AZ_DIAG_HIP_LIB=$L AZ_V9_STAGGER=$sg timeout -k 10 200 python3 tools/net_bench.py --game gomoku15 --batch 2048 --iters 6 --precision f16x3 > $O/c3_$sg.$r.txt 2>&1 || { tail -3 $O/c3_$sg.$r.txt; exit 1; }
    echo "C3 stagger $sg: $(tail -1 $O/c3_$sg.$r.txt | cut -c1-110)"
  done
done
for sg in 0 16000 32000; do
  AZ_DIAG_HIP_LIB=$L AZ_V9_STAGGER=$sg timeout -k 10 200 python3 tools/net_bench.py --game go19 --batch 1024 --iters 6 --precision f16x3 > $O/c4_$sg.txt 2>&1 || { tail -3 $O/c4_$sg.txt; exit 1; }
  echo "C4 stagger $sg: $(tail -1 $O/c4_$sg.txt | cut -c1-110)"
done
AZ_DIAG_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2prof -o run -- python3 bench.py --config c2 --steps 2 --warmup 1 --cpu-baseline 0 --parity-steps 0 > $O/c2prof.json 2> $O/c2prof.err || { tail -5 $O/c2prof.err; exit 1; }
f=$(find $O/c2prof -name "*kernel_stats.csv" | head -1); python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:6]:
    print(f'{r["Name"][:70]:72s} {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f} us {float(r["Percentage"]):6.2f} %')
PY
