# rocprofv3 --pmc progress of searches sized for 400 / 800 simulations (tools/pmc_progress.py): each
# pass killed at 120 s; the first failure ends the run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmchang2}
mkdir -p $O
for cfg in ${CFGS:-400:200 800:200 800:800}; do
  c=${cfg%:*}; r=${cfg#*:}
  t0=$SECONDS
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c${c}r${r} -o run -- python3 tools/pmc_progress.py --games 256 --cap-sims $c --run-sims $r > $O/c${c}r${r}.log 2>&1
  rc=$?
  echo "capacity $c sims, ran $r: rc $rc, $((SECONDS - t0)) s; $(grep -E ' s  ' $O/c${c}r${r}.log | tail -2 | tr '\n' '|')"
  [ $rc -ne 0 ] && break
done
exit 0
