# Round 3 final check on the committed tree: full GPU suite, smoke, the default bench line (C3 +
# parity_mode + CPU baseline), C3 under rocprofv3 --kernel-trace --stats, the C2 bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=25 > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('c3', round(d['value'],2), 'pos/s', round(d['ms_per_step'],1), 'ms/step', d['roofline']['kernel'], round(d['roofline']['frac'],4), 'parity', d.get('parity_mode',{}).get('value'), 'cpu', d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --cpu-baseline 0 --parity-steps 0 --steps 1 --warmup 1 > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $O/trace.log; exit 1; }
grep '"metric"' $O/trace.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c3 under rocprof', round(d['value'],2), round(d['roofline']['avg_launch_ms'],4), 'ms/launch in-bench')"
python3 - <<'PY'
import csv, glob, os
O = os.environ.get("TAG", "final")
f = glob.glob(f"gpurun_out/{O}/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):6.2f} %")
PY
timeout -k 10 300 python3 bench.py --config c2 --cpu-baseline 0 --parity-steps 0 --steps 3 > $O/bench_c2.json 2> $O/bench_c2.err || { echo C2_FAIL; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', round(d['value'],1), 'pos/s', d['roofline']['kernel'], round(d['roofline']['frac'],4))"
