#!/bin/bash
# Submit one gpurun call, resubmitting only while the pool has no free slot or box (gpurun's
# "nothing was charged" transient: no part of the command ran). Any other outcome -- success, a
# failing command, a refusal -- is returned as is, never retried.
#   tools/gpurun_wait.sh LOGFILE TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -qE 'nothing was charged|status=transient' "$LOG" && ! grep -q 'status=ok' "$LOG"; then
    sleep 120
    continue
  fi
  exit $rc
done
exit $rc
