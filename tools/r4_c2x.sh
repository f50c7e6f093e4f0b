#!/bin/bash
# f16x3 FC heads (k_fc_heads_x3<2>): trained-scale / trunk-scaled parity; C2 bench with parity_mode;
# the conv3x3_v9x3 phase timeline (stamp build)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/c2x
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_trained_scale.py -k "f16x3" > $O/net.log 2>&1 || { grep -E "FAIL|Error|assert" $O/net.log | head; tail -5 $O/net.log; exit 1; }
grep -E "f16x3|passed|failed" $O/net.log | tail -30
$T 400 python -u bench.py --config c2 --steps 3 --warmup 1 --cpu-baseline 0 --parity-steps 2 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]);pm=d.get('parity_mode',{})
print('C2', d['value'], d['ms_per_step'], d['roofline']['avg_forward_ms'], 'parity', pm.get('value'), pm.get('ms_per_step'), pm.get('roofline',{}).get('avg_forward_ms'))
print(json.dumps(d['tree_kernels'])[:300])"
AZ_DIAG_HIP_LIB=$PWD/alphazero-multi-game_amd/build_stamps/libaz_hip.so $T 300 python3 -u tools/v9_stamps.py --precision f16x3 > $O/v9_stamps.txt 2>&1 || { tail -5 $O/v9_stamps.txt; exit 1; }
cat $O/v9_stamps.txt
AZ_DIAG_HIP_LIB=$PWD/alphazero-multi-game_amd/build_stamps/libaz_hip.so $T 300 python3 -u tools/v9_stamps.py --precision f16x3 --launch 20 > $O/v9_stamps_first.txt 2>&1 || { tail -5 $O/v9_stamps_first.txt; exit 1; }
cat $O/v9_stamps_first.txt
