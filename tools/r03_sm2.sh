# Round 3: k_smallnet rewrite -- bitwise parity with the round-2 kernel, C2 net parity, A/B timing,
# phase stamps of the new kernel, the C2 bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sm2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -x -q --timeout 120 --timeout-method thread -k "smallnet or trunk_kernel_name or matches_fp32 or position" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert|Mismatch" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python3 tools/net_bench.py --channels 64 --blocks 6 --batch 256 --iters 20 --rounds 4 --sm-kernels 0:8,3:8,2:8 > $O/nb.txt 2>&1; cat $O/nb.txt
for k in 3; do echo "== kernel $k"; AZ_SM_KERNEL=$k timeout -k 10 60 python3 tools/sm_stamps.py 256; echo "-- inner"; AZ_SM_KERNEL=$k SM_INNER=1 timeout -k 10 60 python3 tools/sm_stamps.py 256; done > $O/stamps.txt 2>&1; cat $O/stamps.txt
timeout -k 10 300 python bench.py --config c2 --cpu-baseline 0 --steps 3 > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', round(d['value'],1), 'pos/s', round(d['ms_per_step'],2), 'ms/step', d['roofline']['kernel'], round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms']*1e3,2),'us/conv-equiv')"
AZ_TREE_STAMPS=137 timeout -k 10 120 python3 tools/tree_stamps.py > $O/tree_stamps.txt 2>&1; cat $O/tree_stamps.txt
