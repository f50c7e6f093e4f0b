#!/bin/bash
# --streams A/B (bench.py StreamWorkload): C2 (256 games), the C4 128-game shard and C3, one vs
# several concurrent device handles on one GPU.  Each run under its own limit, && chained.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-streams}
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 300 python3 bench.py --cpu-baseline 0 --parity-steps 0 "$@" > $O/$tag.json 2> $O/$tag.err &&
        python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],2), d['config']['parallelism'])"; }
run c2_s1 --config c2 --steps 20 --warmup 3 &&
run c2_s2 --config c2 --steps 20 --warmup 3 --streams 2 &&
run c2_s4 --config c2 --steps 20 --warmup 3 --streams 4 &&
run c4g128_s1 --config c4 --global-games 128 --steps 8 --warmup 2 &&
run c4g128_s2 --config c4 --global-games 128 --steps 8 --warmup 2 --streams 2 &&
run c3_s1 --steps 4 --warmup 2 &&
run c3_s2 --steps 4 --warmup 2 --streams 2
