# Kernel stats of the C2 bench and the N=8 C3 shard (256 games) under rocprofv3, then the plain C3 bench line.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r02f}
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
for r in rows[:16]:
    print(f'{r["Name"][:70]:70s} calls {int(r["Calls"]):7d} avg {float(r["AverageNs"])/1e3:9.2f} us {float(r["Percentage"]):6.2f}%')
PY
  python3 -c "import json;d=json.load(open('$O/bench_${n}_under_rocprof.json'));print('$n', round(d['value'],1), 'pos/s', round(d['ms_per_step'],1), 'ms/step')"
}
prof c2 300 --config c2 --steps 2 --warmup 1
prof g256 300 --games 256 --steps 2 --warmup 1
timeout -k 10 600 python bench.py --cpu-baseline 0 > $O/bench_c3.json 2> $O/bench_c3.err || { echo BENCH_FAIL; tail -20 $O/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3', round(d['value'],2), 'pos/s', round(d['ms_per_step'],1), 'ms/step', d['roofline']['kernel'], round(d['roofline']['frac'],4))"
