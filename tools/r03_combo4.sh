# Round 3: the rocprofv3 --pmc hang probe in bench.py's own sequence (selfplay step, profiling
# on/off), then the 15x15 v7 tile geometries at C3 (SLIM default, DENSE flag 8, PAD flag 0x400).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/combo4
timeout -k 10 300 python3 tools/net_bench.py --batch 2048 --iters 6 --rounds 3 --flags 0x204,0x20c,0x604 > gpurun_out/combo4/nb_c3_geo.txt 2>&1; cat gpurun_out/combo4/nb_c3_geo.txt
TAG=combo4/pmchang CFGS="256:800:0:step:0 256:800:0:step:1 512:800:0:step:1 2048:800:0:step:1" bash tools/pmc_hang_probe2.sh
# k_smallnet phase stamps per diagnostic variant (NW = 4 kernel; stamps = DV + 1): 1 normal,
# 2 no per-tap barriers, 3 no MFMAs, 5 no fragment reads, 8 no weight DMA, 7 neither reads nor DMA
export AZ_SM_WAVES=4
VARIANTS="1 2 3 5 8 7" timeout -k 10 400 bash tools/sm_diag.sh > gpurun_out/combo4/sm_diag.txt 2>&1; cat gpurun_out/combo4/sm_diag.txt
