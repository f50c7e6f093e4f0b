# k_smallnet (fused 64-filter forward): net parity, batch independence, C2 replay, trained scale, C2 bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sm
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -v -s -k "64 or position_independent or trunk_kernel" --timeout 200 --timeout-method thread > $O/pytest_net.log 2>&1 || { echo NET_FAIL; grep -E "FAILED|Error|error|assert" $O/pytest_net.log | head -20; tail -5 $O/pytest_net.log; exit 1; }
grep -E "dlogit|passed|failed" $O/pytest_net.log | head
timeout -k 10 300 python -u -m pytest tests/test_gpu_selfplay_net.py tests/test_gpu_trained_scale.py -v -s -k "c2" --timeout 200 --timeout-method thread > $O/pytest_c2.log 2>&1 || { echo C2_FAIL; grep -E "FAILED|Error|assert" $O/pytest_c2.log | head -20; tail -5 $O/pytest_c2.log; exit 1; }
grep -E "dlogit|PASSED|passed|failed" $O/pytest_c2.log | head
timeout -k 10 400 python bench.py --config c2 --steps 3 --cpu-baseline 0 > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
