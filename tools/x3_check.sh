#!/bin/bash
# conv3x3_v7x3 (AZ_PREC_BF16X3 on the g8 hi / lo planes): net parity on every geometry + trained
# scale, then trunk timing at the C3 batch (and the fp16 trunk on the same box for reference).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-x3a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_trained_scale.py -x -v -s -k "${X3K:-bf16x3 or trunk_kernel or x3}" --timeout 200 --timeout-method thread > $O/pytest_net.log 2>&1 || { echo NET_FAIL; grep -E 'max\||FAIL|Error|error' $O/pytest_net.log | tail -30; tail -5 $O/pytest_net.log; exit 1; }
grep -E 'dlogit|passed|failed' $O/pytest_net.log | tail -30
for p in ${X3P:-bf16x3 fp16}; do
  timeout -k 10 300 python3 tools/net_bench.py --precision $p --batch ${X3B:-2048} --iters ${X3I:-6} > $O/nb_$p.txt 2>&1 || { echo NB_FAIL; tail -5 $O/nb_$p.txt; exit 1; }
  cat $O/nb_$p.txt
done
