#!/bin/bash
# small-batch DENSE tiles for conv3x3_v7 (128 / 64-row tiles): bitwise vs conv3x3_v6, then the
# C4 / C5 per-rank shard batches (128 boards) per tile size; then the tree PMC at the C3 tree config
# (2048 games x 800 sims, BLOCKS=2) with the clock-stamp timing ON (round 3 needed it off)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/sb
mkdir -p $O
L=$PWD/alphazero-multi-game_amd/build_dev/libaz_hip.so
AZ_DIAG_HIP_LIB=$L timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv_v7.py -k v7_bitwise > $O/bitwise.log 2>&1 || { grep -E "FAIL|Error|assert" $O/bitwise.log | head; tail -5 $O/bitwise.log; exit 1; }
tail -1 $O/bitwise.log
for g in go19 chess; do
  for fl in 0x204 0x804 0x10804 0x20804 0x30804; do
    AZ_DIAG_HIP_LIB=$L AZ_CONV_FLAGS=$fl timeout -k 10 200 python3 tools/net_bench.py --game $g --batch 128 --iters 10 > $O/${g}_$fl.txt 2>&1 || { tail -3 $O/${g}_$fl.txt; exit 1; }
    echo "$g B=128 flags $fl: $(tail -1 $O/${g}_$fl.txt | cut -c1-100)"
  done
done
for fl in 0x204 0x804; do
  AZ_DIAG_HIP_LIB=$L AZ_CONV_FLAGS=$fl timeout -k 10 200 python3 tools/net_bench.py --game go19 --batch 256 --iters 10 > $O/go19_256_$fl.txt 2>&1 || { tail -3 $O/go19_256_$fl.txt; exit 1; }
  echo "go19 B=256 flags $fl: $(tail -1 $O/go19_256_$fl.txt | cut -c1-100)"
done
CONFIG=c3 BLOCKS=2 KT=1 TAG=r4m/tree_c3b2 PMC_TIMEOUT=300 timeout -k 10 900 tools/tree_pmc.sh > $O/tree.log 2>&1 || { tail -8 $O/tree.log; exit 1; }
tail -25 $O/tree.log
