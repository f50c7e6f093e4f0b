#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=1000 FILES="tests/test_gpu_search.py tests/test_gpu_go.py tests/test_gpu_selfplay_net.py tests/test_gpu_host_api.py tests/test_gpu_api.py tests/test_gpu_callback_eval.py tests/test_torchscript.py tests/test_gpu_randwire.py" bash tools/gpu_tests.sh &&
for r in 1 2; do
  for lib in build_head build; do
    AZ_DIAG_HIP_LIB=$R/alphazero-multi-game_amd/$lib/libaz_hip.so timeout -k 10 200 python3 bench.py --config c2 --steps 4 --warmup 1 --cpu-baseline 0 --parity-steps 1 > $O/c2_$lib.$r.json 2> $O/c2_$lib.$r.err || exit 1
    echo "$lib $r $(cut -c60-120 $O/c2_$lib.$r.json)"
  done
done
