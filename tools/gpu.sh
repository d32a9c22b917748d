#!/bin/bash
# Run one command on the GPU box via gpurun; re-submit only when the box never
# ran it (status "transient" with no run time: the box failed while being
# prepared, nothing charged) or no box was free (exit 3).  A command that ran
# -- and failed, or whose box was taken away afterwards -- is never retried.
# Usage: tools/gpu.sh TIMEOUT 'command'
to=$1; shift
for attempt in $(seq 1 ${GPU_SH_ATTEMPTS:-8}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@"
  rc=$?
  read -r st run <<<"$(python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print(d.get('status',''), d.get('run_s') or 0)" 2>/dev/null)"
  if { [ "$rc" = "3" ] || [ "$st" = "transient" ]; } && python3 -c "import sys; sys.exit(0 if float('${run:-0}') == 0 else 1)"; then
    echo "[gpu.sh] box not available (rc=$rc status=$st), attempt $attempt; waiting"
    sleep ${GPU_SH_SLEEP:-60}
    continue
  fi
  exit $rc
done
exit 3
