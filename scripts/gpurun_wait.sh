#!/bin/bash
# Runs one gpurun call, re-submitting it only while the pool reports no free slot or box
# ("transient": nothing ran, nothing was charged).  Any other outcome — success, a failure of the
# command itself, a refusal — ends the loop.  Usage: gpurun_wait.sh <timeout_s> <log> <command>
TMO="$1"; LOG="$2"; shift 2
for attempt in $(seq 1 ${GPURUN_ATTEMPTS:-60}); do
  timeout $((TMO + 900)) /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$@" > "$LOG" 2>&1
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('$(dirname "$0")/../gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ "$st" = "transient" ]; then
    echo "attempt $attempt: no slot, waiting" >> "$LOG.attempts"
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
