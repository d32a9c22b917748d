#!/bin/bash
# Round 5: the flush server's early read of the next position (PRE, the
# product) against the round-4 poll (A/B build, TASX_SRV_PRE=0), alternating
# in one call: checksum and TX segment slots at 1 x 1, 8 x 3, 8 x 7; then the
# timing form of both (TASX_SRV_DIAG), and what each costs device-resident work.  Usage: bash tools/server_pre_ab.sh TAG [ROUNDS]
set -u
TAG=$1; ROUNDS=${2:-3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
AB=$PWD/tas_amd/_lib/libtasx_ab.so
timeout -k 10 300 python -u -m pytest tests/test_server.py tests/test_c_boundary.py -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_server.log" 2>&1 || { echo "server tests failed"; tail -30 "$O/pytest_server.log"; exit 1; }
tail -1 "$O/pytest_server.log"
leg() {  # form: prints one JSON line per shape
  timeout -k 10 150 python3 -u -c "
import json, torch
from tas_amd import benchloop, xsum
xsum.lib()
dev = torch.cuda.current_device()
r = {'form': '$1', 'round': $2}
for th, q in ((1, 1), (8, 3), (8, 7)):
    r[f'csum_{th}x{q}'] = benchloop.fastpath_mt(dev, 8, th, q, 3000, 'server')
    r[f'txseg_{th}x{q}'] = benchloop.txseg_server_mt(dev, 8, th, q, 3000)
print(json.dumps(r), flush=True)
"
}
for i in $(seq 1 "$ROUNDS"); do
  leg pre "$i" >> "$O/ab.jsonl" 2>> "$O/ab.err" || { echo "pre leg failed"; tail "$O/ab.err"; exit 1; }
  TASX_LIB=$AB TASX_SRV_PRE=0 leg poll "$i" >> "$O/ab.jsonl" 2>> "$O/ab.err" || { echo "poll leg failed"; tail "$O/ab.err"; exit 1; }
  tail -2 "$O/ab.jsonl" | cut -c1-400
done
for pre in 1 0; do
  TASX_LIB=$AB TASX_SRV_DIAG=1 TASX_SRV_PRE=$pre leg "diag_pre$pre" 0 >> "$O/diag.jsonl" 2>> "$O/diag.err" || { echo "diag leg failed"; tail "$O/diag.err"; exit 1; }
done
grep server_diag "$O/diag.err" > "$O/diag_sums.jsonl" || true
cat "$O/diag_sums.jsonl"
# what each form costs device-resident work beside it (bench.py server_cost)
price() {
  timeout -k 10 200 python3 -u -c "
import json, sys, threading, time, bench
from tas_amd import xsum
def beat():
    while True:
        time.sleep(20); print('alive', time.time(), file=sys.stderr, flush=True)
threading.Thread(target=beat, daemon=True).start()
xsum.lib()
print(json.dumps({'form': '$1', 'server_cost': bench.server_cost_leg(0, 16)}), flush=True)
"
}
price pre >> "$O/price.jsonl" 2>> "$O/price.err" || { echo "price pre failed"; tail "$O/price.err"; exit 1; }
TASX_LIB=$AB TASX_SRV_PRE=0 price poll >> "$O/price.jsonl" 2>> "$O/price.err" || { echo "price poll failed"; tail "$O/price.err"; exit 1; }
cut -c1-600 "$O/price.jsonl"
