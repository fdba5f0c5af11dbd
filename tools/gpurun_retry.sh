#!/bin/bash
# gpurun with retries ONLY for infrastructure events where the command never ran
# (status=transient / no box free); a command that ran is never re-run.
# usage: tools/gpurun_retry.sh <timeout> '<command>'
T=$1; shift
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" > /tmp/gpurun_last.out 2>&1; rc=$?
  if grep -q "status=transient\|backing off\|no box\|no slot" /tmp/gpurun_last.out && ! grep -q "status=ok" /tmp/gpurun_last.out; then
    echo "[retry $i] $(grep -o 'status=[a-z]*' /tmp/gpurun_last.out | head -1)"; sleep 45; continue
  fi
  break
done
tail -3 /tmp/gpurun_last.out
exit $rc
