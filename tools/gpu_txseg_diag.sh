#!/bin/bash
# Round 5, VERDICT r04 item 4: where a TX segment slot's time goes.  The A/B
# build's timing form of the server (TASX_SRV_DIAG=1: per batch, detection ->
# rows' sums, sums -> stores acknowledged and the done word, the gap to the
# next detection), TX segment slots of 20 and 41 segments, 2 and 4
# workgroups per ring, 1 x 1 and 8 x 3; the checksum slots beside them.
# Usage: bash tools/gpu_txseg_diag.sh TAG
set -u
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
AB=$PWD/tas_amd/_lib/libtasx_ab.so
for k in 2 4; do
  for m in 20 41; do
    TASX_SRV_K=$k TASX_SRV_SEGMAX=$m TASX_SRV_DIAG=1 TASX_LIB=$AB timeout -k 10 120 python3 -u -c "
import json, torch
from tas_amd import benchloop, xsum
xsum.lib()
dev = torch.cuda.current_device()
for th, q in ((1, 1), (8, 3), (8, 7)):
    print(json.dumps({'k': $k, 'segmax': $m, 'shape': f'{th}x{q}', 'txseg': benchloop.txseg_server_mt(dev, 8, th, q, 3000)}), flush=True)
    if $m == 41:
        print(json.dumps({'k': $k, 'shape': f'{th}x{q}', 'csum': benchloop.fastpath_mt(dev, 8, th, q, 3000, 'server')}), flush=True)
" >> "$O/diag.jsonl" 2>> "$O/diag.err" || { echo "failed k=$k m=$m"; tail "$O/diag.err"; exit 1; }
  done
done
grep server_diag "$O/diag.err" > "$O/diag_sums.jsonl" || true
cat "$O/diag.jsonl" "$O/diag_sums.jsonl"
