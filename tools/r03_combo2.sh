# Round 3: host-API tests of the tree-keeping setters and SearchGroup, the object-per-game bench,
# then the rocprofv3 --pmc hang probe (last: its passes are killed at 200 s).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/combo2
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_api.py -v -k "keep_the_tree or search_group or rng" --timeout 200 --timeout-method thread > gpurun_out/combo2/host.log 2>&1; tail -5 gpurun_out/combo2/host.log
timeout -k 10 300 python3 tools/group_bench.py --games 64 --moves 2 > gpurun_out/combo2/group_bench.json 2> gpurun_out/combo2/group_bench.err; cat gpurun_out/combo2/group_bench.json; tail -3 gpurun_out/combo2/group_bench.err
TAG=combo2/pmchang bash tools/pmc_hang_probe.sh
