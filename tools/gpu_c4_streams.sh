#!/bin/bash
# C4: N = 1 (1024 games) and the 8-GPU shard (128 games) with 1-4 concurrent device handles, one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-c4streams}
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 400 python3 bench.py --config c4 --cpu-baseline 0 --parity-steps 0 "$@" > $O/$tag.json 2> $O/$tag.err &&
        python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],2), d['config']['parallelism'], d['config']['games_per_gpu'])"; }
run c4_g1024_s1 --steps 4 --warmup 2 &&
run c4_g128_s1 --global-games 128 --steps 10 --warmup 2 &&
run c4_g128_s2 --global-games 128 --steps 10 --warmup 2 --streams 2 &&
run c4_g128_s3 --global-games 128 --steps 10 --warmup 2 --streams 3 &&
run c4_g128_s4 --global-games 128 --steps 10 --warmup 2 --streams 4 &&
run c4_g1024_s2 --steps 4 --warmup 2 --streams 2
