# Round 3: (1) is the --pmc hang tied to the number of HIP events a search records?  one 800-sim
# selfplay step, profiling on, events on every 64th step (13 tree + 13 net event pairs) vs every
# 16th (the default, hangs); (2) tree PMC at the bench config (tools/tree_pmc.sh, counter passes
# without events); (3) k_smallnet inner stamps of layer 5 (per tap, epilogue) for the normal kernel
# and the no-fragment-read + no-DMA variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/combo5
mkdir -p $O
AZ_PROF_EVERY=64 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pe64 -o run -- python3 tools/pmc_progress.py --games 256 --cap-sims 800 --mode step --profile 1 > $O/pe64.log 2>&1
echo "prof_every 64: rc $? $(grep -E '^ +[0-9.]+ s  ' $O/pe64.log | tail -2 | tr '\n' '|')"
export AZ_HIP_LIB=$PWD/alphazero-multi-game_amd/build_smdiag/libaz_hip.so AZ_SM_WAVES=4 SM_INNER=1
for v in 1 7; do echo "== variant $v"; AZ_SM_STAMPS=$v timeout -k 10 60 python3 tools/sm_stamps.py 256; done > $O/sm_inner.txt 2>&1; cat $O/sm_inner.txt
unset AZ_HIP_LIB AZ_SM_WAVES SM_INNER
TAG=combo5/tree PMC_TIMEOUT=300 timeout -k 10 900 bash tools/tree_pmc.sh > $O/tree.txt 2>&1; echo "tree_pmc rc $?"; tail -60 $O/tree.txt
