#!/bin/bash
# conv3x3_v9x3 (bf16x3 full-width tile): bitwise vs conv3x3_v7x3, oracle geometries, then a same-box
# A/B of the C3 / C4 trunk launch time (conv flag 0x10000000 selects v7x3).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_conv_v7.py -k v9x3 tests/test_gpu_net.py::test_gpu_trunk_kernel_name > gpurun_out/x3w_tests.log 2>&1 || { tail -30 gpurun_out/x3w_tests.log; exit 1; }
tail -3 gpurun_out/x3w_tests.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_net.py -k "bf16x3" > gpurun_out/x3w_net.log 2>&1 || { tail -30 gpurun_out/x3w_net.log; exit 1; }
tail -3 gpurun_out/x3w_net.log
timeout -k 10 300 python -u tools/net_bench.py --precision bf16x3 --batch 2048 --iters 3 --rounds 4 --flags 0x204,0x10000204 2>&1 | tee gpurun_out/x3w_ab_c3.txt
timeout -k 10 300 python -u tools/net_bench.py --game go19 --precision bf16x3 --batch 1024 --iters 3 --rounds 3 --flags 0x204,0x10000204 2>&1 | tee gpurun_out/x3w_ab_c4.txt
