#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=600 FILES="tests/test_gpu_conv_v7.py" K="v7_bitwise" bash tools/gpu_tests.sh &&
timeout -k 10 200 python3 tools/net_bench.py --game go19 --batch 128 --iters 10 --flags 0x204,0x20204,0xa0204 > $O/go19_128.txt 2>&1 && tail -4 $O/go19_128.txt &&
timeout -k 10 200 python3 tools/net_bench.py --game go19 --batch 256 --iters 10 --flags 0x204,0x20204,0xa0204 > $O/go19_256.txt 2>&1 && tail -4 $O/go19_256.txt &&
timeout -k 10 200 python3 tools/net_bench.py --game chess --batch 128 --iters 10 --flags 0x204,0x80204 > $O/chess_128.txt 2>&1 && tail -3 $O/chess_128.txt &&
AZ_STAMPS_GO=1 AZ_TREE_STAMPS=77 timeout -k 10 200 python3 tools/tree_stamps.py 128 800 3 > $O/go_stamps.txt 2>&1 && cat $O/go_stamps.txt
