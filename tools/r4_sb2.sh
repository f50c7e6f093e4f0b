#!/bin/bash
# small-batch routing (DENSE boards < 1024 on conv3x3_v7 small tiles): net parity / bitwise suites on
# the dev build, the C5 / C4 shard-sized forwards; then the --pmc progress probe with timing on / off
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/sb2
mkdir -p $O
L=$PWD/alphazero-multi-game_amd/build_dev/libaz_hip.so
AZ_DIAG_HIP_LIB=$L timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_net.py tests/test_gpu_conv_v7.py > $O/net.log 2>&1 || { grep -E "FAIL|Error|assert" $O/net.log | head; tail -5 $O/net.log; exit 1; }
tail -1 $O/net.log
for g in chess:128 chess:256 chess:1024 go19:128 go19:256 go19:512; do
  IFS=: read gm b <<< "$g"
  AZ_DIAG_HIP_LIB=$L timeout -k 10 200 python3 tools/net_bench.py --game $gm --batch $b --iters 10 > $O/${gm}_$b.txt 2>&1 || { tail -3 $O/${gm}_$b.txt; exit 1; }
  echo "$gm B=$b: $(tail -1 $O/${gm}_$b.txt | cut -c1-100)"
done
AZ_DIAG_HIP_LIB=$L TAG=sb2/pmchang CFGS="256:800:0:step:0 256:800:0:step:1 256:100:0:step:1" timeout -k 10 500 tools/pmc_hang_probe2.sh 2>&1 | tail -20
