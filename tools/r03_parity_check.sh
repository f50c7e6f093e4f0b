# Round 3: the C3 full-size bf16x3 replay (trained-scale heads) and the default bench line with its
# parity_mode object (bf16x3, 1 + 1 moves), without the CPU baseline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03p}
mkdir -p $O
[ -n "$SKIP_REPLAY" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_selfplay_net.py -x -v -s -k "bf16x3" --timeout 380 --timeout-method thread > $O/pytest_x3replay.log 2>&1 || { echo REPLAY_FAIL; tail -30 $O/pytest_x3replay.log; exit 1; }
[ -n "$SKIP_REPLAY" ] || grep -E "trained-scale|passed|failed" $O/pytest_x3replay.log | tail -3
t0=$SECONDS
timeout -k 10 600 python bench.py --cpu-baseline 0 ${BENCH_ARGS:-} > $O/bench_c3.json 2> $O/bench_c3.err || { echo BENCH_FAIL; tail -20 $O/bench_c3.err; exit 1; }
echo "bench wall $((SECONDS - t0)) s"
python3 -c "
import json;d=json.load(open('$O/bench_c3.json'))
print('c3', round(d['value'],2), 'pos/s', round(d['ms_per_step'],1), 'ms/step', d['roofline']['kernel'], round(d['roofline']['frac'],4))
p=d['parity_mode'];print('parity', round(p['value'],2), 'pos/s', round(p['ms_per_step'],1), 'ms/step', p['roofline']['kernel'], round(p['roofline']['avg_launch_ms'],4), 'ms', round(p['roofline']['frac'],4), round(p['roofline']['mfma_issue_frac'],4))"
