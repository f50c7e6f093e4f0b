#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/sb3
mkdir -p $O
L=$PWD/alphazero-multi-game_amd/build_dev/libaz_hip.so
AZ_DIAG_HIP_LIB=$L timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv_v7.py -k v7_bitwise > $O/bitwise.log 2>&1
grep -E "differing \[[0-9]|passed|failed" $O/bitwise.log | tail -8
AZ_DIAG_HIP_LIB=$L timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv_v7.py -k "v7_bitwise and 130" > $O/bitwise130.log 2>&1
grep -E "differing|passed|failed" $O/bitwise130.log | tail -4
