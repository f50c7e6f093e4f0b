#!/bin/bash
# conv3x3_v9x3 variants: bitwise vs conv3x3_v7x3, then a same-box A/B of the C3 / C4 launch time
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv_v7.py -k v9x3 > gpurun_out/x3v_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/x3v_tests.log | head; tail -5 gpurun_out/x3v_tests.log; exit 1; }
tail -1 gpurun_out/x3v_tests.log
$T 400 python -u tools/net_bench.py --precision bf16x3 --batch 2048 --iters 3 --rounds 3 --flags 0x204,0x20000204,0x40000204,0x60000204,0x10000204 2>&1 | tee gpurun_out/x3v_ab_c3.txt || exit 1
$T 300 python -u tools/net_bench.py --game go19 --precision bf16x3 --batch 1024 --iters 3 --rounds 3 --flags 0x204,0x20000204,0x10000204 2>&1 | tee gpurun_out/x3v_ab_c4.txt || exit 1
$T 200 python -u tools/net_bench.py --precision bf16x3 --channels 64 --blocks 6 --batch 256 --iters 30 2>&1 | tee gpurun_out/x3v_c2.txt || exit 1
$T 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_net.py tests/test_gpu_trained_scale.py -k "not fp16_overflow" > gpurun_out/x3v_net.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/x3v_net.log | head; tail -5 gpurun_out/x3v_net.log; exit 1; }
grep -E "dlogit|passed|failed" gpurun_out/x3v_net.log | tail -30
$T 400 python -u bench.py --config c2 --steps 3 --warmup 1 --cpu-baseline 0 --parity-steps 2 > gpurun_out/x3v_bench_c2.json 2> gpurun_out/x3v_bench_c2.err || { tail -5 gpurun_out/x3v_bench_c2.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/x3v_bench_c2.json').read().strip().splitlines()[-1]);print(d['value'], d.get('parity_mode',{}).get('value'), d['roofline']['avg_forward_ms'])"
