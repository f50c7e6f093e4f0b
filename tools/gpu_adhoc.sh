#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=500 FILES="tests/test_gpu_conv_v7.py tests/test_gpu_poison.py tests/test_gpu_net.py" bash tools/gpu_tests.sh &&
timeout -k 10 300 python3 tools/net_bench.py --game gomoku15 --batch 1024 --iters 8 --flags 0x204,0x304 > $O/g15_1024.txt 2>&1 && grep flags= $O/g15_1024.txt &&
timeout -k 10 300 python3 tools/net_bench.py --game go19 --batch 512 --iters 8 --flags 0x204,0x1204 > $O/go19_512.txt 2>&1 && grep flags= $O/go19_512.txt &&
timeout -k 10 300 python3 bench.py --config c4 --global-games 512 --cpu-baseline 0 --parity-steps 0 > $O/c4_g512.json 2> $O/c4_g512.err &&
python3 -c "import json; d=json.loads(open('$O/c4_g512.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c4 games 512', round(d['value'],2), r.get('kernel','')[:40], r.get('avg_launch_ms'))"
