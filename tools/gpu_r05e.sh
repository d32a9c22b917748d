#!/bin/bash
# Round 5: the 41-segment TX slots and the server-price leg.  Usage: bash tools/gpu_r05e.sh TAG [legs-only]
set -u
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
if [ "${2:-}" != "legs-only" ]; then
timeout -k 10 300 python -u -m pytest tests/test_server.py tests/test_c_boundary.py -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_server.log" 2>&1 || { echo "server tests failed rc=$?"; tail -30 "$O/pytest_server.log"; exit 1; }
tail -3 "$O/pytest_server.log"
fi
timeout -k 10 400 python -u -c "
import json, sys, threading, time, bench, torch
from tas_amd import xsum
def beat():
    while True:
        time.sleep(20); print('alive', time.time(), file=sys.stderr, flush=True)
threading.Thread(target=beat, daemon=True).start()
xsum.lib()
print(json.dumps({'server_cost': bench.server_cost_leg(0, 16)}), flush=True)
print(json.dumps({'fastpath_mt': bench.fastpath_mt_leg(3000)}), flush=True)
" > "$O/legs.jsonl" 2> "$O/legs.err" || { echo "legs failed"; tail -20 "$O/legs.err"; exit 1; }
cat "$O/legs.jsonl"
