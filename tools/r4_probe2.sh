#!/bin/bash
# --pmc selfplay-step probe on the round-3 library (build_head) vs the current one
set -o pipefail
cd "$(dirname "$0")/.."
AZ_DIAG_HIP_LIB=$PWD/alphazero-multi-game_amd/build_head/libaz_hip.so TAG=probe5h CFGS="256:800:0:step:0" timeout -k 10 200 tools/pmc_hang_probe2.sh 2>&1 | grep -v "^  File\|^Thread\|^Timeout" | tail -4
