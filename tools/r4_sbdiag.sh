#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/sbdiag
mkdir -p $O
L=$PWD/alphazero-multi-game_amd/build_dev/libaz_hip.so
for B in 130 13 64; do AZ_DIAG_HIP_LIB=$L timeout -k 10 200 python3 -u tools/sb_diag.py $B > $O/b$B.txt 2>&1 || { tail -5 $O/b$B.txt; exit 1; }; echo "B=$B"; cat $O/b$B.txt; done
