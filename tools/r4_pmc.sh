#!/bin/bash
# Round-4 PMC passes: the f16x3 trunk (conv3x3_v9x3<.., f16>, C3 B = 2048) and the tree kernels at the
# C3 bench config (tools/tree_pmc.sh, device clock-stamp timing on).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4m
O=gpurun_out/r4m
T="timeout -k 10"
GAME=gomoku15 BATCH=2048 $T 700 tools/pmc_conv.sh f16x3 r4_f16x3 > $O/pmc_f16x3.log 2>&1 || { tail -5 $O/pmc_f16x3.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_r4_f16x3 --kernel conv3x3_v9x3 --precision f16x3 --out $O/r04_f16x3_v9x3_trunk_pmc.json || exit 1
CONFIG=c3 BLOCKS=20 TAG=r4m/tree_c3 PMC_TIMEOUT=300 $T 1000 tools/tree_pmc.sh > $O/tree_c3.log 2>&1 || { tail -5 $O/tree_c3.log; exit 1; }
tail -30 $O/tree_c3.log
