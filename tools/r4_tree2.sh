#!/bin/bash
# tree-kernel PMC at the C3 bench config (2048 games, 800 sims; BLOCKS trunk blocks, default 2: the
# 20-block move crashes the profiler, SIGSEGV), clock-stamp timing on,
# host sync every 100 simulation steps (the --pmc stall fix)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4m
CONFIG=c3 BLOCKS=${BLOCKS:-2} KT=1 SYNC=100 TAG=r4m/tree_c3s PMC_TIMEOUT=400 timeout -k 10 1100 tools/tree_pmc.sh > gpurun_out/r4m/tree_c3s.log 2>&1 || { tail -8 gpurun_out/r4m/tree_c3s.log; exit 1; }
tail -40 gpurun_out/r4m/tree_c3s.log
