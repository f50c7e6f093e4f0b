#!/bin/bash
# conv3x3_v7: bitwise against v6, net parity, trunk timing v7 vs v6 (15x15, C3 net) at the per-GPU
# batches of 1/2/4/8 GPUs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-v7a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_v7.py -x -q --timeout 120 --timeout-method thread > $O/pytest_v7.log 2>&1; rc=$?
tail -5 $O/pytest_v7.log
if [ $rc -ne 0 ]; then grep -E 'max\||Error|error|assert' $O/pytest_v7.log | head -30; exit 1; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_trained_scale.py -x -q -s --timeout 200 --timeout-method thread > $O/pytest_net.log 2>&1 || { echo NET_FAIL; grep -E 'max\||FAIL|Error' $O/pytest_net.log | tail -30; exit 1; }
grep -E 'dlogit|passed|failed' $O/pytest_net.log | tail -30
for b in 2048 256; do
  timeout -k 10 300 python3 tools/net_bench.py --batch $b --iters 10 --rounds 3 --flags ${NBFLAGS:-0x204,0x604,0x304,0x20c} > $O/nb_$b.txt 2>&1 || { echo NB_FAIL; tail -5 $O/nb_$b.txt; exit 1; }
  cat $O/nb_$b.txt
done
