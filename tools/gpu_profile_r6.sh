#!/bin/bash
# Round-6 profile batch: PMC passes of the C3 trunk kernels (fp16 conv3x3_v7, F16X3 conv3x3_v9x3;
# tools/pmc_conv.sh), the rocprofv3 kernel-trace summary of a default bench run (the roofline's
# kernels, headline + parity_mode), then the tree PMC at one sync per 100 simulation steps with the
# crash reporter on (the round-5 profiler SIGSEGV; tools/tree_pmc.sh).  Each step under its own limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6prof
# geometry A/Bs (conv flag sets, alternating rounds): 15x15 C3 SLIM (default 0x204) vs DENSE (0x20c);
# the C4 128-board shard's tiles: 128-row 3-slot ring (default) vs 64-row (0x30204) vs 64-row 3-slot (0xb0204)
${SKIP_AB:+true} timeout -k 10 300 python3 tools/net_bench.py --game gomoku15 --batch 2048 --flags 0x204,0x20c --rounds 3 --iters 6 > gpurun_out/r6prof/c3_geo_ab.txt 2>&1 &&
${SKIP_AB:+true} timeout -k 10 300 python3 tools/net_bench.py --game go19 --batch 128 --flags 0x204,0x30204,0xb0204 --rounds 3 --iters 20 > gpurun_out/r6prof/c4s_tile_ab.txt 2>&1 &&
${SKIP_PMC:+true} bash tools/pmc_conv.sh fp16 r6_fp16 &&
${SKIP_PMC:+true} bash tools/pmc_conv.sh f16x3 r6_f16x3 &&
${SKIP_TRACE:+true} timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6prof/trace -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/r6prof/bench.json 2> gpurun_out/r6prof/bench.err &&
echo "profile steps ok" &&
{ [ -n "$SKIP_TREE" ] || SYNC=${SYNC:-100} TAG=r6tree bash tools/tree_pmc.sh; }
