#!/bin/bash
# Round-2 API additions on the GPU: reference API scripts, callback evaluator, host API, search regression.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-api}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_callback_eval.py tests/test_gpu_host_api.py tests/test_gpu_search.py tests/test_gpu_go.py -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E 'PASSED|FAILED|ERROR|passed|failed' $O/pytest.log | tail -60
exit $rc
