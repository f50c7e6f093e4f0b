# Round 3: SearchGroup bench (gather window), v7 vs v6 on the DENSE boards (C4 Go 19x19, C5 chess 8x8),
# then the rocprofv3 --pmc progress probe (last: passes killed at 120 s).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/combo3
timeout -k 10 300 python3 tools/group_bench.py --games 64 --moves 2 > gpurun_out/combo3/group_bench.json 2> gpurun_out/combo3/group_bench.err; cat gpurun_out/combo3/group_bench.json; tail -2 gpurun_out/combo3/group_bench.err
timeout -k 10 300 python3 tools/net_bench.py --game go19 --batch 1024 --iters 6 --rounds 3 --flags 0x204,0x4 > gpurun_out/combo3/nb_go19.txt 2>&1; cat gpurun_out/combo3/nb_go19.txt
timeout -k 10 300 python3 tools/net_bench.py --game chess --batch 1024 --iters 6 --rounds 3 --flags 0x204,0x4 > gpurun_out/combo3/nb_chess.txt 2>&1; cat gpurun_out/combo3/nb_chess.txt
TAG=combo3/pmchang2 bash tools/pmc_hang_probe2.sh
