# Round-1 v6 measurement: default bench line, the bench under rocprofv3 kernel trace, trunk PMC passes.
set -e
export TMPDIR=/tmp
O=gpurun_out/r01_v6
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --cpu-baseline 0 --steps 1 --warmup 1 > $O/bench_under_rocprof.json 2> $O/rocprof.err
bash tools/pmc_conv.sh fp16 v6
python3 tools/pmc_summary.py gpurun_out/pmc_v6 --kernel conv3x3_v6 --out $O/trunk_pmc.json > /dev/null
echo all-done
