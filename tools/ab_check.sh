#!/bin/bash
# Parity of the trunk paths + same-process A/B of conv flag sets on the C3 / C4 / C5 nets.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for g in ${GAMES:-gomoku15 go19 chess}; do
  timeout -k 10 200 python3 tools/net_bench.py --game $g --batch ${BATCH:-2048} --flags $FLAGS --iters 5 --rounds 4 > $O/nb_$g.txt 2>&1 || { echo NB_FAIL $g; tail -5 $O/nb_$g.txt; exit 1; }
  echo $g; cat $O/nb_$g.txt
done
