#!/bin/bash
# k_smallnet: net parity (incl. the C2 replay and trained-scale C2), the 4- vs 8-wave block timing
# (phase stamps of block 0), then the C2 bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-smc}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_trained_scale.py tests/test_gpu_selfplay_net.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in 4 8; do echo "== $w waves"; AZ_SM_WAVES=$w timeout -k 10 60 python3 tools/sm_stamps.py 256 | sed -n '1,3p;13,17p'; done
timeout -k 10 300 python bench.py --config c2 --cpu-baseline 0 --steps 3 > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', round(d['value'],1), 'pos/s', round(d['ms_per_step'],2), 'ms/step', d['roofline']['kernel'], round(d['roofline']['frac'],4))"
