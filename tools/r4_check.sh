#!/bin/bash
# Round-4 GPU check: the new / changed GPU tests, then same-box timing (bf16x3 trunk A/B, C2 parity
# forward, fp16 range-guard A/B against the committed build_head library).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
$T 600 $PYT tests/test_gpu_net.py > gpurun_out/r4_net.log 2>&1 || { tail -40 gpurun_out/r4_net.log; exit 1; }
tail -2 gpurun_out/r4_net.log
$T 900 $PYT -s tests/test_gpu_trained_scale.py tests/test_gpu_dataset.py tests/test_batch_queue.py > gpurun_out/r4_ts.log 2>&1 || { tail -40 gpurun_out/r4_ts.log; exit 1; }
grep -E "max\|dlogit|passed|failed" gpurun_out/r4_ts.log | tail -30
$T 300 python -u tools/net_bench.py --precision bf16x3 --batch 2048 --iters 3 --rounds 3 --flags 0x204,0x10000204 2>&1 | tee gpurun_out/r4_x3_ab_c3.txt || exit 1
$T 300 python -u tools/net_bench.py --game go19 --precision bf16x3 --batch 1024 --iters 3 --rounds 3 --flags 0x204,0x10000204 2>&1 | tee gpurun_out/r4_x3_ab_c4.txt || exit 1
$T 120 python -u tools/net_bench.py --precision bf16x3 --channels 64 --blocks 6 --batch 256 --iters 30 2>&1 | tee gpurun_out/r4_c2x3.txt || exit 1
ABTAG=r4_guard_c3 ROUNDS=3 $T 400 tools/ab_builds.sh || exit 1
ABTAG=r4_guard_c2 ROUNDS=3 NBARGS="--channels 64 --blocks 6 --batch 256 --iters 30" $T 300 tools/ab_builds.sh || exit 1
$T 400 python -u bench.py --config c2 --steps 3 --warmup 1 --cpu-baseline 0 --parity-steps 2 > gpurun_out/r4_bench_c2.json 2> gpurun_out/r4_bench_c2.err || { tail -5 gpurun_out/r4_bench_c2.err; exit 1; }
tail -c 1500 gpurun_out/r4_bench_c2.json
