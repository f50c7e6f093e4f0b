set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6j; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 300 python3 bench.py --cpu-baseline 0 --parity-steps 0 "$@" > $O/$tag.json 2> $O/$tag.err &&
        python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],2), d['config']['parallelism'], d['config']['games_per_gpu'])"; }
run c3_g256_s1 --global-games 256 --steps 8 --warmup 2 &&
run c3_g256_s2 --global-games 256 --steps 8 --warmup 2 --streams 2 &&
run c3_g256_s1b --global-games 256 --steps 8 --warmup 2 &&
run c3_g256_s2b --global-games 256 --steps 8 --warmup 2 --streams 2 &&
run c3_g512_s1 --global-games 512 --steps 6 --warmup 2 &&
run c3_g512_s2 --global-games 512 --steps 6 --warmup 2 --streams 2 &&
run c3_g1024_s2 --global-games 1024 --steps 4 --warmup 2 --streams 2
