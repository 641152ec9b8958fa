#!/bin/bash
# Submit one gpurun call; resubmit ONLY when no box was free / the call never ran
# (gpurun's "transient" status: nothing charged, no part of the command ran), at
# most TRIES times, SLEEP seconds apart. Any call that ran — pass or fail — is final.
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1 to=$2 cmd=$3
for i in $(seq 1 ${TRIES:-6}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  if grep -q "status=transient" "$log" && grep -q "run 0.0s\|run Nones" "$log"; then
    echo "[retry $i: no box]" >> "$log.tries"
    sleep ${SLEEP:-150}
    continue
  fi
  break
done
