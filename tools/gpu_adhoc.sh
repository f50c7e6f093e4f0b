#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=1000 FILES="tests/test_gpu_go.py tests/test_gpu_dataset.py tests/test_gpu_host_api.py" bash tools/gpu_tests.sh &&
timeout -k 10 300 python3 bench.py --config c4 --global-games 128 --steps 3 --warmup 1 --cpu-baseline 0 --parity-steps 2 > $O/bench_c4_g128.json 2> $O/bench_c4_g128.err && cut -c1-200 $O/bench_c4_g128.json &&
timeout -k 10 400 python3 bench.py --config c4 --steps 2 --warmup 1 --cpu-baseline 0 --parity-steps 1 > $O/bench_c4.json 2> $O/bench_c4.err && cut -c1-200 $O/bench_c4.json
