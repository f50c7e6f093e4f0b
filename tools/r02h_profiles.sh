# Round-2 final profile set: C3 bench under rocprofv3 --kernel-trace --stats (trunk average vs the
# in-bench HIP events), then the tree-kernel PMC over a full 800-sim C3 move (tools/tree_pmc.sh).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r02h}
O=gpurun_out/$T
mkdir -p $O
if [ -z "$SKIP_C3" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_c3 -o run -- python3 bench.py --cpu-baseline 0 --steps 1 --warmup 1 > $O/bench_c3_under_rocprof.json 2> $O/bench_c3_prof.err || { echo PROF_FAIL; tail -8 $O/bench_c3_prof.err; exit 1; }
cp $(find $O/tr_c3 -name "*kernel_stats.csv" | head -1) $O/bench_c3_kernel_stats.csv
python3 tools/trace_gaps.py $O/tr_c3 > $O/bench_c3_trace_gaps.txt
fi
TAG=$T/tree bash tools/tree_pmc.sh
