#!/bin/bash
# Net parity + per-kernel times of the C3 forward (B = 2048) under rocprofv3 kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/qp
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/net_bench.py --iters 5 > $O/nb.log 2>&1 || { echo PROF_FAIL; tail -5 $O/nb.log; exit 1; }
tail -1 $O/nb.log
f=$(find $O/trace -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:60]:60s} calls {int(r["Calls"]):6d} avg {float(r["AverageNs"])/1e3:9.1f} us  {float(r["Percentage"]):6.2f}%')
PY
