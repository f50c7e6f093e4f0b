# Kernel stats of the C2 bench, the N=8 shard (256 games per GPU) and the C3 bench under rocprofv3.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r02d}
O=gpurun_out/$T
mkdir -p $O
prof() {  # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$n -o run -- python3 bench.py --cpu-baseline 0 "$@" > $O/bench_${n}_under_rocprof.json 2> $O/bench_$n.err || { echo PROF_FAIL $n; grep -v "^    @" $O/bench_$n.err | tail -8; exit 1; }
  cp $(find $O/tr_$n -name "*kernel_stats.csv" | head -1) $O/bench_${n}_kernel_stats.csv
  python3 - $O/bench_${n}_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:18]:
    print(f'{r["Name"][:70]:70s} calls {int(r["Calls"]):7d} avg {float(r["AverageNs"])/1e3:9.2f} us {float(r["Percentage"]):6.2f}%')
PY
  cat $O/bench_${n}_under_rocprof.json
}
prof c2 300 --config c2 --steps 2 --warmup 1
prof g256 300 --games 256 --steps 2 --warmup 1
prof c3 400 --steps 1 --warmup 1 ${C3ARGS}
