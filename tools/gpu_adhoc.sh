#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
#   FILES   GPU test files to run first;  AB=1: same-box A/B of build_head vs build (tools/ab_builds.sh)
#   BENCH=0 skips the driver-config bench
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=600 FILES="${FILES:-tests/test_gpu_search.py tests/test_gpu_callback_eval.py}" bash tools/gpu_tests.sh &&
{ [ -z "$AB" ] || ABTAG=${TAG:-adhoc}/ab ROUNDS=${ROUNDS:-3} bash tools/ab_builds.sh; } &&
{ [ "${BENCH:-1}" = 0 ] || { timeout -k 10 590 python3 bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} > $O/bench_c3.json 2> $O/bench_c3.err && tail -c 600 $O/bench_c3.json; }; }
