#!/bin/bash
# AZ_PREC_F16X3 (fp16 hi / lo pieces): net parity, trained-scale / trunk-scaled errors, v9x3 == v7x3
# bitwise, fp16-piece range guard, then the C3 / C2 split-precision forwards' timing (net_bench)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/f16x3
T="timeout -k 10"
O=gpurun_out/f16x3
$T 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_trained_scale.py \
    tests/test_gpu_net.py > $O/net.log 2>&1 || { grep -E "FAIL|Error|assert" $O/net.log | head; tail -5 $O/net.log; exit 1; }
grep -E "trunk-scaled|: \|logit|c[2-5] (f16x3|bf16x3|fp16)|passed|failed" $O/net.log | tail -60
$T 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv_v7.py -k v9x3 \
    > $O/v9.log 2>&1 || { grep -E "FAIL|Error|assert" $O/v9.log | head; tail -5 $O/v9.log; exit 1; }
tail -2 $O/v9.log
for prec in f16x3 bf16x3; do
  $T 200 python3 tools/net_bench.py --game gomoku15 --batch 2048 --iters 6 --precision $prec > $O/nb_c3_$prec.txt 2>&1 || { tail -3 $O/nb_c3_$prec.txt; exit 1; }
  echo "C3 $prec $(tail -1 $O/nb_c3_$prec.txt | cut -c1-150)"
  $T 200 python3 tools/net_bench.py --channels 64 --blocks 6 --batch 256 --iters 30 --precision $prec > $O/nb_c2_$prec.txt 2>&1 || { tail -3 $O/nb_c2_$prec.txt; exit 1; }
  echo "C2 $prec $(tail -1 $O/nb_c2_$prec.txt | cut -c1-150)"
done
