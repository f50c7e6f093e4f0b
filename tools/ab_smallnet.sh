# Same-box A/B of two library builds (default: the C2 net, B = 256; NBARGS overrides the net_bench arguments): build_ab (the committed kernel) vs
# build (the working tree), alternating, ROUNDS times each; tools/net_bench.py forward timing.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${ABTAG:-smab}
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-4}); do
  for lib in build_ab build; do
    AZ_DIAG_HIP_LIB=$PWD/alphazero-multi-game_amd/$lib/libaz_hip.so timeout -k 10 120 python3 tools/net_bench.py --game gomoku15 ${NBARGS:---channels 64 --blocks 6 --batch 256 --iters 30} > $O/$lib.$r.txt 2>&1 || { echo FAIL $lib; tail -3 $O/$lib.$r.txt; exit 1; }
    echo "$lib $(tail -1 $O/$lib.$r.txt | cut -c1-100)"
  done
done
