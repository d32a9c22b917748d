#!/bin/bash
# Run one command on the GPU box via gpurun; re-submit only when the box never
# ran it (status "transient": the box failed while being prepared, nothing
# charged) or no box was free (exit 3).  A command that ran and failed is never
# retried.  Usage: tools/gpu.sh TIMEOUT 'command'
to=$1; shift
for attempt in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$rc" = "3" ] || [ "$st" = "transient" ]; then
    echo "[gpu.sh] box not available (rc=$rc status=$st), attempt $attempt; waiting"
    sleep 60
    continue
  fi
  exit $rc
done
exit 3
