# Round-1 final measurement (conv v6 padded 15x15 / DENSE other boards, nt epilogue, LDS pool):
# trunk PMC passes (C3 and C4 nets), then the C3 bench line, the C3 bench under rocprofv3 kernel
# trace, and the C4 Go bench line.  Summaries go to gpurun_out/r01c (copied into profiles/).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r01c}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pmc-c3
bash tools/pmc_conv.sh fp16 c3 > $O/pmc_c3.log 2>&1 || { echo FAIL pmc-c3; tail -5 $O/pmc_c3.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_c3 --kernel conv3x3_v6 --out $O/${TAG:-r01c}_fp16_v6_trunk_pmc.json > /dev/null || { echo FAIL sum-c3; exit 1; }
step pmc-go19
GAME=go19 BATCH=1024 bash tools/pmc_conv.sh fp16 go19 > $O/pmc_go19.log 2>&1 || { echo FAIL pmc-go19; tail -5 $O/pmc_go19.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_go19 --kernel conv3x3_v6 --game go19 --board 19 --boards 1024 --out $O/${TAG:-r01c}_go19_fp16_v6_trunk_pmc.json > /dev/null || { echo FAIL sum-go19; exit 1; }
cp $O/${TAG:-r01c}_*_trunk_pmc.json profiles/
step bench-c3
timeout -k 10 600 python bench.py > $O/${TAG:-r01c}_bench.json 2> $O/bench.err || { echo FAIL bench; tail -5 $O/bench.err; exit 1; }
cat $O/${TAG:-r01c}_bench.json
step rocprof-c3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --cpu-baseline 0 --steps 1 --warmup 1 > $O/${TAG:-r01c}_bench_under_rocprof.json 2> $O/rocprof.err || { echo FAIL rocprof; tail -5 $O/rocprof.err; exit 1; }
cp $(find $O/trace -name "*kernel_stats.csv" | head -1) $O/${TAG:-r01c}_bench_kernel_stats.csv
step bench-go
timeout -k 10 600 python bench.py --game go --steps 1 --warmup 1 > $O/${TAG:-r01c}_go_c4_bench.json 2> $O/bench_go.err || { echo FAIL go; tail -5 $O/bench_go.err; exit 1; }
cat $O/${TAG:-r01c}_go_c4_bench.json
step done
