# conv3x3_v8 (one block per 256-row tile x 256 channels) against conv3x3_v6 bitwise, the network
# suite against the fp32 reference, then a trunk A/B against v7 (flag 0x20000) at the C3 batch.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03v8}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_v7.py tests/test_gpu_net.py > $O/tests.log 2>&1 &&
tail -3 $O/tests.log &&
timeout -k 10 240 python -u tools/net_bench.py --batch 2048 --flags 0x204,0x20204 --rounds 4 > $O/ab.log 2>&1 &&
tail -12 $O/ab.log
