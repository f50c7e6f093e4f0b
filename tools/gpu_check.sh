#!/bin/bash
# Round GPU check: dataset tests, the full GPU suite, smoke, default bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/chk
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dataset.py -x -v -s --timeout 200 --timeout-method thread > $O/pytest_ds.log 2>&1 || { echo DS_FAIL; tail -40 $O/pytest_ds.log; exit 1; }
grep -E "extract|passed|failed" $O/pytest_ds.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
