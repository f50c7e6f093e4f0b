#!/bin/bash
# Net parity + trunk timing per board + the default C3 bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/qc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_selfplay_net.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for g in gomoku15 go19 chess; do
  timeout -k 10 200 python3 tools/net_bench.py --game $g --batch 2048 --iters 10 > $O/nb_$g.txt 2>&1 || { echo NB_FAIL $g; tail -5 $O/nb_$g.txt; exit 1; }
  cat $O/nb_$g.txt
done
if [ "${WITH_BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py --cpu-baseline 0 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench.json'));print('C3', round(d['value'],2), 'pos/s', round(d['roofline']['avg_launch_ms'],4), 'ms/launch', round(d['roofline']['frac'],4))"
fi
