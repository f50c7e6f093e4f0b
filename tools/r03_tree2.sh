# Round 3: tree-kernel latency, second cut (one TreeDev argument, root-header record hint, VGPR lane
# broadcasts): the search parity tests, tree stamps at C2, the C2 bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tree2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_api.py tests/test_gpu_host_api.py tests/test_gpu_go.py "tests/test_gpu_selfplay_net.py::test_gpu_c2_full_size_replay" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert|Mismatch" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
AZ_TREE_STAMPS=137 timeout -k 10 120 python3 tools/tree_stamps.py > $O/tree_stamps.txt 2>&1; cat $O/tree_stamps.txt
for i in 1 2; do timeout -k 10 300 python bench.py --config c2 --cpu-baseline 0 --parity-steps 0 --steps 3 > $O/bench_c2_$i.json 2> $O/bench_c2.err || { echo BENCH_FAIL; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2_$i.json'));print('c2', round(d['value'],1), 'pos/s', round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['avg_launch_ms']*1e3,2),'us/conv-equiv', {k: round(v['avg_launch_us'],2) for k, v in d['tree_kernels'].items() if isinstance(v, dict)})"; done
