set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r01_fp16
timeout -k 10 600 python bench.py > gpurun_out/r01_fp16/bench.json 2> gpurun_out/r01_fp16/bench.err
cat gpurun_out/r01_fp16/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01_fp16/trace -o run -- python3 bench.py --cpu-baseline 0 --steps 1 --warmup 1 > gpurun_out/r01_fp16/bench_under_rocprof.json 2> gpurun_out/r01_fp16/rocprof.err
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r01_fp16/fetch -o run -- python3 tools/net_bench.py --precision fp16 --iters 3 > /dev/null 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r01_fp16/write -o run -- python3 tools/net_bench.py --precision fp16 --iters 3 > /dev/null 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r01_fp16/sq -o run -- python3 tools/net_bench.py --precision fp16 --iters 3 > /dev/null 2>&1
echo all-done
