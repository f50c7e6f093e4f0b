# What makes an 800-sim C3 move hang under rocprofv3 --pmc (round 2: killed at 90 s and 500 s; 100-
# and 400-sim moves finish in seconds)?  Not the dispatch count: tools/pmc_limit.sh ran 13k
# dispatches under --pmc in 2 s.  Here one move of the bench under one FETCH_SIZE pass, growing the
# device footprint (node pools ~ games x sims, TT 24 MB per game): 512 / 1024 games at 800 sims,
# then 2048 at 600 and 800.  Each pass is killed at 200 s; the first failure ends the run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmchang}
mkdir -p $O
( while sleep 30; do echo "pass running ($(date +%T))"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for cfg in ${CFGS:-512:800 1024:800 2048:600 2048:800}; do
  g=${cfg%:*}; s=${cfg#*:}
  t0=$SECONDS
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/g${g}s${s} -o run -- python3 bench.py --cpu-baseline 0 --parity-steps 0 --steps 1 --warmup 0 --sims $s --blocks 2 --games $g > $O/g${g}s${s}.log 2>&1
  rc=$?
  nd=$(cat $(find $O/g${g}s${s} -name '*counter_collection.csv' 2>/dev/null) /dev/null | grep -c FETCH_SIZE || true)
  echo "games $g sims $s: rc $rc, $((SECONDS - t0)) s, $nd counter rows; $(grep -o '"value": [0-9.]*' $O/g${g}s${s}.log | head -1)"
  [ $rc -ne 0 ] && break
done
exit 0
