#!/bin/bash
# product build check after the FC / stagger changes: net parity subset, C2 bench (+ parity_mode),
# then the PMC passes (tools/r4_pmc.sh)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_net.py tests/test_gpu_conv_v7.py -k "smallnet or trunk_kernel or c3_net or x3 or v9x3" > $O/net.log 2>&1 || { grep -E "FAIL|Error|assert" $O/net.log | head; tail -5 $O/net.log; exit 1; }
tail -1 $O/net.log
$T 400 python -u bench.py --config c2 --steps 3 --warmup 1 --cpu-baseline 0 --parity-steps 2 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]);pm=d.get('parity_mode',{})
print('C2', d['value'], d['ms_per_step'], d['roofline']['avg_forward_ms'], 'parity', pm.get('value'), pm.get('ms_per_step'), pm.get('roofline',{}).get('avg_forward_ms'))"
tools/r4_pmc.sh
