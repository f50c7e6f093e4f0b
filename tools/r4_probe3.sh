#!/bin/bash
# --pmc selfplay-step probe with the step's phase trace (where the host thread stops)
set -o pipefail
cd "$(dirname "$0")/.."
AZ_STEP_TRACE=1 AZ_DIAG_HIP_LIB=$PWD/alphazero-multi-game_amd/build_dev/libaz_hip.so TAG=probe6 CFGS="256:800:0:step:0" timeout -k 10 200 tools/pmc_hang_probe2.sh 2>&1 | grep -v "^  File\|^Thread\|^Timeout" | tail -3
grep "^\[step\]" gpurun_out/probe6/g256c800r0stepp0.log | tail -12
