#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=600 FILES="tests/test_gpu_go.py tests/test_gpu_dataset.py" bash tools/gpu_tests.sh &&
AZ_STAMPS_GO=1 AZ_TREE_STAMPS=77 timeout -k 10 200 python3 tools/tree_stamps.py 128 800 3 > $O/go_stamps.txt 2>&1 && cat $O/go_stamps.txt &&
timeout -k 10 300 python3 tools/net_bench.py --game go19 --batch 1024 --iters 6 --flags 0x204,0xa0804,0x20804,0x40804,0x10804,0x30804 > $O/go19_1024.txt 2>&1 && grep flags= $O/go19_1024.txt &&
timeout -k 10 300 python3 tools/net_bench.py --game chess --batch 1024 --iters 6 --flags 0x204,0xa0804,0x20804,0x30804 > $O/chess_1024.txt 2>&1 && grep flags= $O/chess_1024.txt &&
timeout -k 10 300 python3 tools/net_bench.py --game gomoku15 --batch 2048 --iters 4 --flags 0x204,0xa0a0c,0x10a0c > $O/g15_2048.txt 2>&1 && grep flags= $O/g15_2048.txt &&
timeout -k 10 400 python3 bench.py --config c4 --global-games 128 --cpu-baseline 0 --parity-steps 0 > $O/bench_c4_g128.json 2> $O/bench_c4_g128.err && tail -c 200 $O/bench_c4_g128.json
