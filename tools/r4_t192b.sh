#!/bin/bash
# product build: the conv / net GPU suites (incl. the forced 192-row tiles, bitwise vs v6), then
# 19x19 / 8x8 small batches per tile size
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/t192b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv_v7.py tests/test_gpu_net.py > $O/suite.log 2>&1 || { grep -E "FAIL|Error|assert" $O/suite.log | head; tail -5 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for g in go19:128 go19:256 chess:128; do
  IFS=: read gm b <<< "$g"
  for fl in 0x204 0x40804 0x20804; do
    AZ_CONV_FLAGS=$fl timeout -k 10 200 python3 tools/net_bench.py --game $gm --batch $b --iters 10 > $O/${gm}_${b}_$fl.txt 2>&1 || { tail -3 $O/${gm}_${b}_$fl.txt; exit 1; }
    echo "$gm B=$b flags $fl: $(tail -1 $O/${gm}_${b}_$fl.txt | cut -c1-80)"
  done
done
