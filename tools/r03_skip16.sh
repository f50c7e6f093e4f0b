# Round 3: conv3x3_v7 SLIM with the dead 16th fragment's MFMAs skipped -- bitwise parity vs v6,
# C3 trunk A/B (flags 0x204 default vs 0x10204 = keep them), then the tree PMC at the C3 games /
# sims with a 2-block trunk (the 20-block counter passes crash the profiler's host thread).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/skip16
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_v7.py tests/test_gpu_net.py -x -q --timeout 200 --timeout-method thread -k "not smallnet" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert|Mismatch" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 tools/net_bench.py --batch 2048 --iters 6 --rounds 4 --flags 0x204,0x10204 > $O/nb.txt 2>&1; cat $O/nb.txt
BLOCKS=2 TAG=skip16/tree PMC_TIMEOUT=200 timeout -k 10 700 bash tools/tree_pmc.sh > $O/tree.txt 2>&1; echo "tree_pmc rc $?"; tail -50 $O/tree.txt
