# A/B of two library builds on the same box: tools/net_bench.py alternately on build_head
# (the committed kernel) and build (the working tree), ROUNDS times each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/abb
mkdir -p $O
G=${GAME:-gomoku15}
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in build_head build; do
    AZ_DIAG_HIP_LIB=$PWD/alphazero-multi-game_amd/$lib/libaz_hip.so timeout -k 10 200 python3 tools/net_bench.py --game $G --batch ${BATCH:-2048} --iters 6 > $O/$lib.$r.txt 2>&1 || { echo FAIL $lib; tail -3 $O/$lib.$r.txt; exit 1; }
    echo "$lib $(tail -1 $O/$lib.$r.txt | cut -c1-90)"
  done
done
