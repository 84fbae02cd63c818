#!/bin/bash
# Submit one gpurun call, re-submitting only while the pod has no free GPU slot (gpurun exit 3 /
# "slot(s) on this pod are busy": nothing ran, nothing was charged). Any other outcome -- the
# command ran, failed, timed out, or was refused -- ends it: a GPU step is never retried here.
#   tools/gpurun_wait.sh LOG TIMEOUT 'command'
log=$1; to=$2; shift 2
for i in $(seq 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "slot(s) on this pod are busy\|status=transient" "$log"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
