#!/bin/bash
# the same probe, dev build, trace off then on
set -o pipefail
cd "$(dirname "$0")/.."
L=$PWD/alphazero-multi-game_amd/build_dev/libaz_hip.so
AZ_DIAG_HIP_LIB=$L TAG=probe7off CFGS="256:800:0:step:0" timeout -k 10 200 tools/pmc_hang_probe2.sh 2>&1 | grep -v "^  File\|^Thread\|^Timeout" | tail -2
AZ_STEP_TRACE=1 AZ_DIAG_HIP_LIB=$L TAG=probe7on CFGS="256:800:0:step:0" timeout -k 10 200 tools/pmc_hang_probe2.sh 2>&1 | grep -v "^  File\|^Thread\|^Timeout" | tail -2
