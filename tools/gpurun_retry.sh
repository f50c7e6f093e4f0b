#!/bin/bash
# gpurun with retries while the pool has no free box or slot (exit code 3, or a "transient" status
# with nothing run and nothing charged); any other outcome -- including a failure of the command
# itself -- is returned at once.  Usage: tools/gpurun_retry.sh OUTFILE TIMEOUT CMD...
OUT=$1; TO=$2; shift 2
for i in $(seq 1 ${RETRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$OUT" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { grep -q "status=transient" "$OUT" && grep -qE "run 0.0s|run Nones|backing off" "$OUT"; }; then
    echo "attempt $i: no box ($(date +%T)), retrying" >> "$OUT.retries"
    sleep ${RETRY_SLEEP:-90}
    continue
  fi
  exit $rc
done
exit 3
