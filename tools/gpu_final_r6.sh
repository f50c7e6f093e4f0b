#!/bin/bash
# Round-6 closing batch on one box: the whole -m gpu suite + smoke, then the per-GPU shard lines of
# the C3 strong-scaling configs (N = 8: 256 games per GPU; N = 2: 1024) next to the N = 1 line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6final}
mkdir -p $O
{ [ -n "$SKIP_SUITE" ] || TAG=${TAG:-r6final}/t LIMIT=900 SMOKE=1 bash tools/gpu_tests.sh; } &&
timeout -k 10 300 python3 bench.py --global-games 256 --steps 8 --warmup 2 --cpu-baseline 0 --parity-steps 0 > $O/bench_c3_g256.json 2> $O/bench_c3_g256.err &&
timeout -k 10 300 python3 bench.py --global-games 1024 --steps 4 --warmup 2 --cpu-baseline 0 --parity-steps 0 > $O/bench_c3_g1024.json 2> $O/bench_c3_g1024.err &&
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --cpu-baseline 0 --parity-steps 0 > $O/bench_c3_g2048.json 2> $O/bench_c3_g2048.err &&
for f in $O/bench_c3_g*.json; do echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['value'],2), d['config']['games_per_gpu'], round(d['roofline']['avg_launch_ms'],4))")"; done
