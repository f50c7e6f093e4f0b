#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=900 SMOKE=1 bash tools/gpu_tests.sh &&
timeout -k 10 560 python3 bench.py > $O/bench_c3.json 2> $O/bench_c3.err && tail -c 200 $O/bench_c3.json && echo &&
timeout -k 10 300 python3 bench.py --config c2 --cpu-baseline 0 > $O/bench_c2.json 2> $O/bench_c2.err && echo c2 ok &&
timeout -k 10 400 python3 bench.py --config c4 --global-games 128 --cpu-baseline 0 > $O/bench_c4_g128.json 2> $O/bench_c4_g128.err && echo c4g128 ok
