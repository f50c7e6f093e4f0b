#!/bin/bash
# Ad hoc GPU measurement batch of the current work item (overwritten as work moves on; the outputs
# that back a number are copied into profiles/).  Every GPU step under its own time limit, && chained.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${TAG:-adhoc}
mkdir -p $O
TAG=${TAG:-adhoc}/t LIMIT=600 FILES="tests/test_gpu_go.py tests/test_gpu_dataset.py tests/test_gpu_api.py tests/test_gpu_host_api.py" bash tools/gpu_tests.sh &&
AZ_STAMPS_GO=1 AZ_TREE_STAMPS=77 timeout -k 10 200 python3 tools/tree_stamps.py 128 800 3 > $O/go_stamps.txt 2>&1 && grep -A4 "k_expand_backup" $O/go_stamps.txt &&
timeout -k 10 400 python3 bench.py --config c4 --global-games 128 --cpu-baseline 0 --parity-steps 0 > $O/c4g128.json 2> $O/c4g128.err &&
python3 -c "import json; d=json.loads(open('$O/c4g128.json').read().strip().splitlines()[-1]); tk=d['tree_kernels']; print('c4g128', round(d['value'],2), {k: round(v['avg_launch_us'],1) for k,v in tk.items() if isinstance(v, dict)})"  &&
timeout -k 10 500 python3 bench.py --global-games 256 --cpu-baseline 0 > $O/c3_g256.json 2> $O/c3_g256.err &&
python3 -c "import json; d=json.loads(open('$O/c3_g256.json').read().strip().splitlines()[-1]); p=d['parity_mode']; print('c3 256', round(d['value'],2), 'parity', round(p.get('value') or 0,2), p.get('steps'), (p.get('roofline') or {}).get('kernel'))"
