#!/bin/bash
# Round 5: frames and shm mapped MTYPE_UC
# (hipExtHostRegisterUncached / hipHostMallocUncached, A/B build TASX_HOST_UC=1)
# so the L2 never caches them, and the server without its per-batch acquire
# (TASX_SRV_ACQ=2).  First whether the server tests see stale lines without
# the acquire on ordinary pinned memory (they must, or they prove nothing),
# then the same on UC memory, then throughput, latency and the price.
# Usage: bash tools/uc_probe.sh TAG
set -u
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
AB=$PWD/tas_amd/_lib/libtasx_ab.so
K="refilled or reused or random_flushes or tx_segments_random"
t() {  # name env... -- pytest; rc 0/1 allowed (a failing test is a finding here)
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -q --timeout 120 --timeout-method thread -k "$K" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 "$O/$name.log")"
  [ $rc -le 1 ] || exit $rc
}
t stale_default TASX_LIB=$AB TASX_SRV_ACQ=2
t uc_noacq TASX_LIB=$AB TASX_HOST_UC=1 TASX_SRV_ACQ=2
t uc_acq TASX_LIB=$AB TASX_HOST_UC=1
leg() {
  env "$@" timeout -k 10 150 python3 -u -c "
import json, torch
from tas_amd import benchloop, xsum
xsum.lib()
dev = torch.cuda.current_device()
r = {}
for th, q in ((1, 1), (8, 3), (8, 7)):
    r[f'csum_{th}x{q}'] = benchloop.fastpath_mt(dev, 8, th, q, 3000, 'server')
    r[f'txseg_{th}x{q}'] = benchloop.txseg_server_mt(dev, 8, th, q, 3000)
print(json.dumps(r), flush=True)
"
}
for i in 1 2; do
  echo "{\"form\": \"product\", \"round\": $i}" >> "$O/legs.jsonl"
  leg X=1 >> "$O/legs.jsonl" 2>> "$O/legs.err" || { echo "leg failed"; tail "$O/legs.err"; exit 1; }
  echo "{\"form\": \"uc_noacq\", \"round\": $i}" >> "$O/legs.jsonl"
  leg TASX_LIB=$AB TASX_HOST_UC=1 TASX_SRV_ACQ=2 >> "$O/legs.jsonl" 2>> "$O/legs.err" || { echo "leg failed"; tail "$O/legs.err"; exit 1; }
  echo "{\"form\": \"uc_acq\", \"round\": $i}" >> "$O/legs.jsonl"
  leg TASX_LIB=$AB TASX_HOST_UC=1 >> "$O/legs.jsonl" 2>> "$O/legs.err" || { echo "leg failed"; tail "$O/legs.err"; exit 1; }
  tail -6 "$O/legs.jsonl" | cut -c1-300
done
timeout -k 10 200 python3 -u tools/price_leg.py product >> "$O/price.jsonl" 2>> "$O/price.err" || { echo "price failed"; tail "$O/price.err"; exit 1; }
TASX_LIB=$AB TASX_HOST_UC=1 TASX_SRV_ACQ=2 timeout -k 10 200 python3 -u tools/price_leg.py uc_noacq >> "$O/price.jsonl" 2>> "$O/price.err" || { echo "price failed"; tail "$O/price.err"; exit 1; }
cut -c1-600 "$O/price.jsonl"
