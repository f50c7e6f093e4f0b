# Round 3: FC heads in one launch (k_fc_heads<PD>) -- net parity (fp32 oracle, batch position
# independence, every precision), the C2 replay and search parity, tree sub-phase stamps, C2 bench,
# C2 kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fc
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_search.py tests/test_gpu_api.py tests/test_gpu_go.py "tests/test_gpu_selfplay_net.py::test_gpu_c2_full_size_replay" tests/test_gpu_trained_scale.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert|Mismatch" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
AZ_TREE_STAMPS=137 timeout -k 10 120 python3 tools/tree_stamps.py > $O/tree_stamps.txt 2>&1; cat $O/tree_stamps.txt
timeout -k 10 300 python bench.py --config c2 --cpu-baseline 0 --parity-steps 0 --steps 3 > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', round(d['value'],1), 'pos/s', round(d['ms_per_step'],2), 'ms/step')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config c2 --cpu-baseline 0 --parity-steps 0 --steps 2 --warmup 1 --kernel-timing 0 > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $O/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/fc/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):6.2f} %")
PY
