#!/bin/bash
# Full GPU suite (no -x) + smoke + bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/full
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | sed 's/.*:://' | tail -60
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
if [ "${WITH_GO:-0}" = 1 ]; then
  timeout -k 10 600 python bench.py --game go --steps 1 --warmup 1 > $O/bench_go.json 2> $O/bench_go.err || { echo GO_BENCH_FAIL; tail -20 $O/bench_go.err; exit 1; }
  cat $O/bench_go.json
fi
