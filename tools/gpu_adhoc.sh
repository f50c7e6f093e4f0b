#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=700 FILES="tests/test_gpu_conv_v7.py tests/test_gpu_poison.py" bash tools/gpu_tests.sh &&
AZ_SB_FLAGS="v6=0x904,v7_128=0x20804,v7_128r3=0xa0804,v7_64=0x30804,v7_192=0x40804" \
  timeout -k 10 120 python3 tools/sb_diag.py 130 > $O/sb19_130.txt 2>&1 &&
timeout -k 10 200 python3 tools/net_bench.py --game go19 --batch 128 --iters 10 --flags 0x204,0x20204,0xa0204 > $O/go19_128.txt 2>&1 && tail -4 $O/go19_128.txt &&
timeout -k 10 200 python3 tools/net_bench.py --game go19 --batch 256 --iters 10 --flags 0x204,0x20204,0xa0204 > $O/go19_256.txt 2>&1 && tail -4 $O/go19_256.txt &&
timeout -k 10 420 python3 bench.py > $O/bench_c3.json 2> $O/bench_c3.err && tail -c 600 $O/bench_c3.json
