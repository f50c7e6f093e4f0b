#!/bin/bash
# final check of the 19x19 small-batch routing: conv / net GPU suites on the product build
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv_v7.py tests/test_gpu_net.py tests/test_gpu_go.py > $O/suite.log 2>&1 || { grep -E "FAIL|Error|assert" $O/suite.log | head; tail -5 $O/suite.log; exit 1; }
tail -1 $O/suite.log
