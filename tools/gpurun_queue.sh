#!/bin/bash
# Sends one GPU call, re-sending it only while the pool reports no free box or slot
# (gpurun status "transient": nothing ran, nothing was charged), up to 12 tries.
#   tools/gpurun_queue.sh LOG TIMEOUT 'COMMAND'
LOG=$1 T=$2 CMD=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  [ "$st" != "transient" ] && break
  sleep 120
done
tail -5 "$LOG"
