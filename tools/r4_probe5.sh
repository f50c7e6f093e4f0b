#!/bin/bash
# --pmc selfplay step with a host sync every N simulation steps (bounded queued dispatches)
set -o pipefail
cd "$(dirname "$0")/.."
L=$PWD/alphazero-multi-game_amd/build_dev/libaz_hip.so
for n in 50 50 200 0; do
  AZ_SYNC_EVERY=$n AZ_STEP_TRACE=1 AZ_DIAG_HIP_LIB=$L TAG=probe8_$n CFGS="256:800:0:step:0" timeout -k 10 200 tools/pmc_hang_probe2.sh 2>&1 | grep -v "^  File\|^Thread\|^Timeout" | tail -1 | sed "s/^/sync every $n: /"
done
