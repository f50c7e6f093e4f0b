#!/bin/bash
# Same-box A/B of two library builds: tools/net_bench.py alternately on each build in LIBS
# (default "build_head build": the committed kernels vs the working tree), ROUNDS times each.
#   NBARGS   net_bench.py arguments (default: the C3 trunk at B = 2048)
#   ABTAG    output directory under gpurun_out/
# e.g. the C2 fused forward: NBARGS="--channels 64 --blocks 6 --batch 256 --iters 30" tools/ab_builds.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${ABTAG:-abb}
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in ${LIBS:-build_head build}; do
    AZ_DIAG_HIP_LIB=$PWD/alphazero-multi-game_amd/$lib/libaz_hip.so timeout -k 10 200 python3 tools/net_bench.py \
        ${NBARGS:---game gomoku15 --batch 2048 --iters 6} > $O/$lib.$r.txt 2>&1 || { echo FAIL $lib; tail -3 $O/$lib.$r.txt; exit 1; }
    echo "$lib $(tail -1 $O/$lib.$r.txt | cut -c1-110)"
  done
done
