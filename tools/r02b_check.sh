# Round-2 check: trained-scale precision figures, the GPU suite, the default bench line and the
# bf16x3 (parity-precision) C3 bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_trained_scale.py -v -s --timeout 200 --timeout-method thread > $O/trained.log 2>&1 || { echo TRAINED_FAIL; tail -40 $O/trained.log; exit 1; }
grep -E "max\|dlogit" $O/trained.log
if [ "${WITH_TESTS:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
fi
timeout -k 10 600 python bench.py --cpu-window 15 > $O/bench_c3.json 2> $O/bench_c3.err || { echo BENCH_FAIL; tail -20 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
timeout -k 10 600 python bench.py --precision bf16x3 --steps 1 --warmup 1 --cpu-baseline 0 > $O/bench_c3_bf16x3.json 2> $O/bench_c3_bf16x3.err || { echo BENCH_FAIL bf16x3; tail -20 $O/bench_c3_bf16x3.err; exit 1; }
cat $O/bench_c3_bf16x3.json
