#!/bin/bash
# GPU test runner: one pytest process (stops at the first failure), each step under its own time
# limit.  FILES (default: the whole tests/ dir), K (pytest -k expression), POISON (AZ_TEST_POISON:
# every net forward runs over poisoned activation buffers, tests/conftest.py), TAG (output dir
# under gpurun_out/), SMOKE=1 also runs __graft_entry__.smoke().
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tests}
mkdir -p $O
[ -n "$POISON" ] && export AZ_TEST_POISON=$POISON
timeout -k 10 ${LIMIT:-900} python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
    ${K:+-k "$K"} > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
if [ -n "$SMOKE" ]; then
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log
fi
