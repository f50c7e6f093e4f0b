# Round-2 GPU check: the GPU suite, the default bench line (C3, strong shard at N=1 = 2048 games,
# CPU baseline), the per-GPU shard sizes of N=2/4/8 (1024/512/256 games) and the C2 workload.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02a}
mkdir -p $O
if [ "${WITH_TESTS:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
fi
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo BENCH_FAIL; tail -20 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
for g in ${SHARDS:-1024 512 256}; do
  timeout -k 10 400 python bench.py --games $g --steps 3 --cpu-baseline 0 > $O/bench_g$g.json 2> $O/bench_g$g.err || { echo BENCH_FAIL $g; tail -20 $O/bench_g$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_g$g.json'));print('G=$g', round(d['value'],2), 'pos/s', round(d['ms_per_step'],1), 'ms/step', round(d['roofline']['avg_launch_ms'],4), 'ms/launch', round(d['roofline']['frac'],4))"
done
timeout -k 10 400 python bench.py --config c2 --steps 3 --cpu-window 15 > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL c2; tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
