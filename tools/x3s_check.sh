#!/bin/bash
# k_smallnet_x3 (C2 in bf16x3) parity + timing; conv3x3_v9x3 vs v7x3 A/B (C3, C4)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu"
$T 300 $PYT tests/test_gpu_net.py -k "smallnet_x3 or trunk_kernel_name" "tests/test_gpu_trained_scale.py::test_gpu_trained_scale_outputs" > gpurun_out/x3s_tests.log 2>&1 || { grep -E "dlogit|FAIL|Error" gpurun_out/x3s_tests.log | head -20; tail -5 gpurun_out/x3s_tests.log; exit 1; }
grep -E "dlogit|passed|failed" gpurun_out/x3s_tests.log
$T 120 python -u tools/net_bench.py --precision bf16x3 --channels 64 --blocks 6 --batch 256 --iters 30 2>&1 | tee gpurun_out/x3s_c2.txt || exit 1
$T 120 python -u tools/net_bench.py --precision fp16 --channels 64 --blocks 6 --batch 256 --iters 30 2>&1 | tee -a gpurun_out/x3s_c2.txt || exit 1
$T 300 python -u tools/net_bench.py --precision bf16x3 --batch 2048 --iters 3 --rounds 3 --flags 0x204,0x10000204 2>&1 | tee gpurun_out/x3s_ab_c3.txt || exit 1
$T 300 python -u tools/net_bench.py --game go19 --precision bf16x3 --batch 1024 --iters 3 --rounds 3 --flags 0x204,0x10000204 2>&1 | tee gpurun_out/x3s_ab_c4.txt || exit 1
