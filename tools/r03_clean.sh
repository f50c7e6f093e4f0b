# Round 3: after removing the smallnet ring variant and the compiled-out diagnostic variants --
# net / conv parity, the smallnet bitwise test, C2 replay, and the C2 line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/clean
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_conv_v7.py tests/test_gpu_trained_scale.py "tests/test_gpu_selfplay_net.py::test_gpu_c2_full_size_replay" tests/test_gpu_go.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py --config c2 --cpu-baseline 0 --parity-steps 0 --steps 3 > $O/bench_c2.json 2> $O/bench_c2.err || { echo C2_FAIL; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', round(d['value'],1), 'pos/s', d['roofline']['kernel'], round(d['roofline']['frac'],4))"
