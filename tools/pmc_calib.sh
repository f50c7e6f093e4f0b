#!/bin/bash
# HBM-counter calibration of the C3 fp16 trunk (conv3x3_v7) per dispatch: which part of the PMC
# read excess over the algorithmic bytes (1.23x, profiles/r06_c3_fp16_trunk_pmc.json) is the
# halo (16-B-per-lane LDS-DMA reads, both channel halves of a tile) and which the residual join of
# every second conv (8-B / 4-B-per-lane buffer loads, widths MI355X_MICROARCH.md leaves
# uncalibrated).  tools/pmc_calib.py splits the dispatches into the two convs of a block.
# Passes (each its own run; TCC slots: FETCH_SIZE 3, 4 per pass):
#   fetch: FETCH_SIZE;  req: TCC_EA0_RDREQ{,_64B,_128B,_DRAM}_sum (request sizes -> bytes)
#   hit (HIT=1): TCC_HIT_sum TCC_MISS_sum;  write, wrreq (WR=1): WRITE_SIZE; TCC_EA0_WRREQ{,_64B}_sum
# LIB: an in-tree build directory (AZ_DIAG_HIP_LIB), default the shipped build/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-calib}
mkdir -p $OUT
[ -n "$LIB" ] && export AZ_DIAG_HIP_LIB=$PWD/alphazero-multi-game_amd/$LIB/libaz_hip.so
NB="python3 tools/net_bench.py --game gomoku15 --batch 2048 --precision ${PREC:-fp16} --iters 2"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $NB > $OUT/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $OUT/req -o run -- $NB > $OUT/req.log 2>&1 &&
{ [ -z "$WR" ] || timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $NB > $OUT/write.log 2>&1; } &&
{ [ -z "$WR" ] || timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/wrreq -o run -- $NB > $OUT/wrreq.log 2>&1; } &&
{ [ -z "$HIT" ] || timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/hit -o run -- $NB > $OUT/hit.log 2>&1; } &&
echo "calib done ${LIB:-build}"
