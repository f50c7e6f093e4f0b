#!/bin/bash
# Round-6 profile batch: PMC passes of the C3 trunk kernels (fp16 conv3x3_v7, F16X3 conv3x3_v9x3;
# tools/pmc_conv.sh), the rocprofv3 kernel-trace summary of a default bench run (the roofline's
# kernels, headline + parity_mode), then the tree PMC at one sync per 100 simulation steps with the
# crash reporter on (the round-5 profiler SIGSEGV; tools/tree_pmc.sh).  Each step under its own limit.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6prof
${SKIP_PMC:+true} bash tools/pmc_conv.sh fp16 r6_fp16 &&
${SKIP_PMC:+true} bash tools/pmc_conv.sh f16x3 r6_f16x3 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6prof/trace -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/r6prof/bench.json 2> gpurun_out/r6prof/bench.err &&
echo "bench under rocprof ok" &&
SYNC=${SYNC:-100} TAG=r6tree bash tools/tree_pmc.sh
