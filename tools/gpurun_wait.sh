#!/bin/bash
# Submit one gpurun call, re-submitting only while gpurun itself reports that nothing ran: exit
# code 3 (no free box / slot; nothing charged). Any other outcome -- the command ran (and passed,
# failed, faulted or timed out), or was refused -- ends it with that exit code: a GPU step is
# never retried here, and the command's own output is never matched.
#   tools/gpurun_wait.sh LOG TIMEOUT 'command'
log=$1; to=$2; shift 2
for i in $(seq 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ]; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
