# Round-2 profiles: C2 replay test, v7 trunk PMC passes (C3), kernel stats of the C3 bench (v7),
# the C2 bench and the N=8 shard (256 games per GPU).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r02c}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_selfplay_net.py -v -k full_size --timeout 250 --timeout-method thread > $O/pytest_full.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_full.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest_full.log
bash tools/pmc_conv.sh fp16 ${T}_v7 || { echo PMC_FAIL; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_${T}_v7 --kernel conv3x3_v7 --out $O/fp16_v7_trunk_pmc.json && cat $O/fp16_v7_trunk_pmc.json
prof() {  # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$n -o run -- python3 bench.py --cpu-baseline 0 "$@" > $O/bench_${n}_under_rocprof.json 2> $O/bench_$n.err || { echo PROF_FAIL $n; tail -20 $O/bench_$n.err; exit 1; }
  cp $(find $O/tr_$n -name "*kernel_stats.csv" | head -1) $O/bench_${n}_kernel_stats.csv
  python3 - $O/bench_${n}_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{r["Name"][:70]:70s} calls {int(r["Calls"]):7d} avg {float(r["AverageNs"])/1e3:9.2f} us {float(r["Percentage"]):6.2f}%')
PY
  cat $O/bench_${n}_under_rocprof.json
}
prof c3 400 --steps 1 --warmup 1
prof c2 300 --config c2 --steps 2 --warmup 1
prof g256 300 --games 256 --steps 2 --warmup 1
