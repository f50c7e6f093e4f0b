#!/bin/bash
# PMC passes over tools/net_bench.py (C3 trunk, B=2048; GAME / BATCH env for other nets): one SQ/GRBM pass, one FETCH_SIZE pass,
# one WRITE_SIZE pass (separate passes, as gfx950's TCC slots require).  Output: gpurun_out/pmc_<tag>/
set -e
PREC=${1:-fp16}; TAG=${2:-$PREC}; GAME=${GAME:-gomoku15}; BATCH=${BATCH:-2048}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/net_bench.py --game $GAME --batch $BATCH --precision $PREC --iters 5 > $OUT/trace.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 tools/net_bench.py --game $GAME --batch $BATCH --precision $PREC --iters 3 > $OUT/sq.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 tools/net_bench.py --game $GAME --batch $BATCH --precision $PREC --iters 3 > $OUT/fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 tools/net_bench.py --game $GAME --batch $BATCH --precision $PREC --iters 3 > $OUT/write.log 2>&1
echo pmc done
