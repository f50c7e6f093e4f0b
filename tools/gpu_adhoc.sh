#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=400 FILES="tests/test_gpu_conv_v7.py" bash tools/gpu_tests.sh &&
for B in 256 512 1024; do
  timeout -k 10 300 python3 tools/net_bench.py --game gomoku15 --batch $B --iters 8 --flags 0x204,0xa04,0xa0a0c,0xb0a0c,0x40a0c,0x10a0c > $O/g15_$B.txt 2>&1 || exit 1
  echo "B=$B"; grep flags= $O/g15_$B.txt
done
