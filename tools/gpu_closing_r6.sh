#!/bin/bash
# Round-6 GPU batch: the whole -m gpu suite + smoke (tools/gpu_tests.sh), the two-rank RCCL probe on
# one GPU (tools/dist_probe.py), then the tree PMC at one sync per 100 simulation steps with the crash
# reporter on (last: a profiler crash ends the call).  Each GPU step under its own limit, && chained.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6close}
mkdir -p $O
{ [ -n "$SKIP_SUITE" ] || TAG=${TAG:-r6close}/t LIMIT=900 SMOKE=1 bash tools/gpu_tests.sh; } &&
{ timeout -k 10 240 python3 tools/dist_probe.py --timeout 60 > $O/dist_probe.txt 2>&1; rc=$?; tail -3 $O/dist_probe.txt;
  [ $rc -le 1 ]; } &&     # 0 pass, 1 a reported failure (e.g. RCCL refusing two ranks on one GPU); a timeout / signal ends the call
{ [ -n "$SKIP_TREE" ] || SYNC=${SYNC:-100} TAG=${TAG:-r6close}/tree bash tools/tree_pmc.sh; }
