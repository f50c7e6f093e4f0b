#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=900 SMOKE=1 bash tools/gpu_tests.sh &&
timeout -k 10 560 python3 bench.py > $O/bench_c3.json 2> $O/bench_c3.err && tail -c 300 $O/bench_c3.json
