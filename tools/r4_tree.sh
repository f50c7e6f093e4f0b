#!/bin/bash
# tree-kernel PMC at the C3 bench config (20 blocks, 2048 games, 800 sims), clock-stamp timing on
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4m
CONFIG=c3 BLOCKS=20 TAG=r4m/tree_c3 PMC_TIMEOUT=300 timeout -k 10 1000 tools/tree_pmc.sh > gpurun_out/r4m/tree_c3.log 2>&1 || { tail -8 gpurun_out/r4m/tree_c3.log; exit 1; }
tail -30 gpurun_out/r4m/tree_c3.log
