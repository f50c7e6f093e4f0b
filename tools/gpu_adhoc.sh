#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=400 FILES="tests/test_gpu_pool_heads.py" bash tools/gpu_tests.sh &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tail -o run -- python3 tools/net_bench.py --game go19 --batch 128 --iters 4 --flags 0x204,0x400204 > $O/prof_tail.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tail15 -o run -- python3 tools/net_bench.py --game gomoku15 --batch 2048 --iters 2 --rounds 2 --flags 0x204,0x400204,0x200204 > $O/prof_tail15.log 2>&1 &&
for r in 1 2; do for f in 204 400204; do
  timeout -k 10 300 python3 bench.py --config c4 --global-games 128 --cpu-baseline 0 --parity-steps 0 --conv-flags $f > $O/c4g128_${f}_$r.json 2> $O/c4g128_${f}_$r.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/c4g128_${f}_$r.json').read().strip().splitlines()[-1]); print('c4g128 $f $r', d['value'])"
done; done &&
for f in 204 400204 200204; do
  timeout -k 10 300 python3 bench.py --cpu-baseline 0 --parity-steps 0 --conv-flags $f > $O/c3_${f}.json 2> $O/c3_${f}.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/c3_${f}.json').read().strip().splitlines()[-1]); print('c3 $f', d['value'])"
done
