#!/bin/bash
# A/B: conv3x3_v9x3 two-burst epilogue (build_dev) vs the committed kernel (build), f16x3 C3 trunk;
# then the C2 bench's per-kernel times (rocprofv3 --kernel-trace --stats)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/ab4
mkdir -p $O
ROUNDS=3 ABTAG=ab4/v9epi LIBS="build build_dev" NBARGS="--game gomoku15 --batch 2048 --iters 6 --precision f16x3" tools/ab_builds.sh || exit 1
ROUNDS=2 ABTAG=ab4/v9epi_go LIBS="build build_dev" NBARGS="--game go19 --batch 1024 --iters 6 --precision f16x3" tools/ab_builds.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2prof -o run -- python3 bench.py --config c2 --steps 2 --warmup 1 --cpu-baseline 0 --parity-steps 0 > $O/c2prof.json 2> $O/c2prof.err || { tail -5 $O/c2prof.err; exit 1; }
f=$(find $O/c2prof -name "*kernel_stats.csv" | head -1); python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{r["Name"][:70]:72s} {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.2f} us {float(r["Percentage"]):6.2f} %')
PY
