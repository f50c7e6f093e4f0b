#!/bin/bash
# rocprofv3 --pmc progress of searches (tools/pmc_progress.py): CFGS entries are
# games:capacity-sims:run-sims:mode:profile; each pass is killed at 120 s; the first failure ends
# the run.  Round 3: --mode sims at 256 games finished at 400 and 800 sims (1-2 s); bench.py itself
# (one selfplay step, 512 games, 800 sims) hung before printing anything.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmchang2}
mkdir -p $O
for cfg in ${CFGS:-256:800:800:sims:0 256:800:0:step:0 256:800:0:step:1}; do
  IFS=: read g c r mode prof <<< "$cfg"
  n=g${g}c${c}r${r}${mode}p${prof}
  t0=$SECONDS
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$n -o run -- python3 tools/pmc_progress.py --games $g --cap-sims $c --run-sims $r --mode $mode --profile $prof > $O/$n.log 2>&1
  rc=$?
  echo "$n: rc $rc, $((SECONDS - t0)) s; $(grep -E '^ +[0-9.]+ s  ' $O/$n.log | tail -2 | tr '\n' '|')"
  [ $rc -ne 0 ] && { grep -A6 'Current thread\|Thread 0x' $O/$n.log | tail -14; break; }
done
exit 0
