#!/bin/bash
# The whole GPU suite, smoke(), then the C2 and C3 bench lines (no profiler).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-rc}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --config c2 --cpu-baseline 0 --steps 3 > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL c2; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', round(d['value'],1), 'pos/s', round(d['ms_per_step'],2), 'ms/step', {k: round(v['avg_launch_us'],2) for k, v in d['tree_kernels'].items() if k != 'note'})"
timeout -k 10 600 python bench.py --cpu-baseline 0 > $O/bench_c3.json 2> $O/bench_c3.err || { echo BENCH_FAIL c3; tail -20 $O/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3', round(d['value'],2), 'pos/s', round(d['ms_per_step'],1), 'ms/step', d['roofline']['kernel'], round(d['roofline']['frac'],4), {k: round(v['avg_launch_us'],2) for k, v in d['tree_kernels'].items() if k != 'note'})"
