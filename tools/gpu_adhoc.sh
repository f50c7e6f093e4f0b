#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
AZ_STEP_TRACE=1 timeout -k 10 200 python3 bench.py --config c2 --steps 3 --warmup 1 --cpu-baseline 0 --parity-steps 0 > $O/bench_c2_trace.json 2> $O/bench_c2_trace.err && cut -c1-200 $O/bench_c2_trace.json &&
TAG=${TAG:-adhoc}/tree20 BLOCKS=20 SYNC=10 PMC_TIMEOUT=300 bash tools/tree_pmc.sh > $O/tree20.txt 2>&1 && tail -40 $O/tree20.txt &&
timeout -k 10 560 python3 bench.py --parity-steps 2 > $O/bench_c3.json 2> $O/bench_c3.err && cut -c1-300 $O/bench_c3.json
