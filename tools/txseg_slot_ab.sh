#!/bin/bash
# Round 5 A/B: TX segments per server slot, 20 (round 4) against 41 (one slot
# per 32-segment flush), alternating processes on one box (libtasx_ab.so,
# TASX_SRV_SEGMAX), 1 x 1, 8 x 3, 8 x 7; with TASX_SRV_DIAG the server's
# per-batch timing sums.  Usage: bash tools/txseg_slot_ab.sh TAG [rounds]
set -u
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
for r in $(seq 1 ${2:-3}); do
  for m in 20 41; do
    TASX_SRV_SEGMAX=$m TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so timeout -k 10 120 python3 -u -c "
import json, torch
from tas_amd import benchloop, xsum
xsum.lib()
dev = torch.cuda.current_device()
out = {'segmax': $m, 'round': $r}
for th, q in ((1, 1), (8, 3), (8, 7)):
    out[f'{th}x{q}'] = benchloop.txseg_server_mt(dev, 8, th, q, 3000)
print(json.dumps(out), flush=True)
" >> "$O/txseg_slots.jsonl" 2>> "$O/txseg_slots.err" || { echo "failed"; tail "$O/txseg_slots.err"; exit 1; }
  done
done
cat "$O/txseg_slots.jsonl"
