#!/bin/bash
# net parity (incl. trained / trunk-scaled, fp16 range guard), C2 bench, then tools/r4_meas.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_net.py tests/test_gpu_trained_scale.py > gpurun_out/c2_net.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/c2_net.log | head; tail -5 gpurun_out/c2_net.log; exit 1; }
grep -E "trunk-scaled|c[2-5] (bf16x3|fp16)|passed|failed" gpurun_out/c2_net.log | tail -40
$T 400 python -u bench.py --config c2 --steps 3 --warmup 1 --cpu-baseline 0 --parity-steps 2 > gpurun_out/c2_bench_c2.json 2> gpurun_out/c2_bench_c2.err || { tail -5 gpurun_out/c2_bench_c2.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/c2_bench_c2.json').read().strip().splitlines()[-1]);print('C2', d['value'], d.get('parity_mode',{}).get('value'), d['roofline']['avg_forward_ms'])"
tools/r4_meas.sh
