# Round 3: C2 under rocprofv3 --kernel-trace --stats (per-kernel averages of the production path,
# kernel timing off), then the tree-kernel PMC at the C2 bench config (tools/tree_pmc.sh CONFIG=c2).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c2prof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config c2 --cpu-baseline 0 --parity-steps 0 --steps 2 --warmup 1 --kernel-timing 0 > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $O/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c2prof/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):6.2f} %")
PY
CONFIG=c2 TAG=c2prof/tree PMC_TIMEOUT=200 timeout -k 10 700 bash tools/tree_pmc.sh > $O/tree.txt 2>&1; echo "tree_pmc rc $?"; tail -45 $O/tree.txt
