#!/bin/bash
# the whole GPU suite + smoke on the product build, the shard-sized forwards, the default bench line,
# then the --pmc progress probe (timing on / off)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/full
mkdir -p $O
TAG=full tools/gpu_suite.sh || exit 1
for g in chess:128 chess:1024 go19:128 go19:256 go19:1024; do
  IFS=: read gm b <<< "$g"
  timeout -k 10 200 python3 tools/net_bench.py --game $gm --batch $b --iters 10 > $O/${gm}_$b.txt 2>&1 || { tail -3 $O/${gm}_$b.txt; exit 1; }
  echo "$gm B=$b: $(tail -1 $O/${gm}_$b.txt | cut -c1-100)"
done
timeout -k 10 600 python -u bench.py > $O/bench_c3_default.json 2> $O/bench_c3_default.err || { tail -5 $O/bench_c3_default.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/bench_c3_default.json').read().strip().splitlines()[-1]);pm=d.get('parity_mode',{})
print('C3', round(d['value'],2), d['roofline']['avg_launch_ms'], 'parity', pm.get('value'), pm.get('roofline',{}).get('avg_launch_ms'), 'cpu', d['cpu_baseline']['value'])"
TAG=full/pmchang CFGS="256:800:0:step:0 256:800:0:step:1 256:100:0:step:1" timeout -k 10 500 tools/pmc_hang_probe2.sh 2>&1 | tail -12
