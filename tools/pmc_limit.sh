#!/bin/bash
# Does rocprofv3 --pmc stop on the dispatch count?  The 800-sim C3 move hung under --pmc (round 2,
# twice) while 100- and 400-sim moves finished.  Here the C3 net's forward (≈46 dispatches at
# batch 16) runs 100 / 170 / 260 times under one SQ counter, each pass killed at 150 s: if the
# passes past ~8k dispatches hang and the shorter ones finish, the limit is the dispatch count.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmclim}
mkdir -p $O
( while sleep 30; do echo "pmc pass running ($(date +%T))"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for n in ${ITERS:-100 170 260}; do
  t0=$SECONDS
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES --output-format csv -d $O/n$n -o run -- python3 tools/net_bench.py --batch 16 --iters $n > $O/n$n.log 2>&1
  rc=$?
  nd=$(cat $(find $O/n$n -name '*counter_collection.csv' 2>/dev/null) /dev/null | grep -c SQ_WAVES || true)
  echo "iters $n: rc $rc, $((SECONDS - t0)) s, $nd counter rows"
  [ $rc -ne 0 ] && break
done
exit 0
