#!/bin/bash
# Tree-kernel parity (every search / Go / host-API / callback / self-play replay test), then the C2
# bench line and a C2 kernel trace under rocprofv3 (per-kernel averages + the inter-kernel gaps).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tc}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_go.py tests/test_gpu_api.py \
  tests/test_gpu_host_api.py tests/test_gpu_callback_eval.py tests/test_gpu_selfplay_net.py -x -v --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --config c2 --cpu-baseline 0 --steps 3 > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', round(d['value'],1), 'pos/s', round(d['ms_per_step'],2), 'ms/step', {k: round(v['avg_launch_us'],2) for k, v in d['tree_kernels'].items() if k != 'note'})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_c2 -o run -- python3 bench.py --config c2 --cpu-baseline 0 --steps 2 > $O/bench_c2_under_rocprof.json 2> $O/bench_c2_prof.err || { echo PROF_FAIL; tail -8 $O/bench_c2_prof.err; exit 1; }
python3 tools/trace_gaps.py $O/tr_c2
