#!/bin/bash
# Round 5, VERDICT r04 item 5: what the resident server costs device-resident
# work, and why.  The server_cost leg with the product's system-scope acquire
# per batch and with the A/B build's agent-scope / no acquire (diagnostics
# only), two alternating rounds; then the product leg under rocprofv3
# --kernel-trace, so the headline kernel's own durations in each state can be
# told from gaps between launches.  Usage: bash tools/server_price.sh TAG
set -u
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
AB=$PWD/tas_amd/_lib/libtasx_ab.so
for i in 1 2; do
  timeout -k 10 200 python3 -u tools/price_leg.py system >> "$O/price.jsonl" 2>> "$O/price.err" || { echo "price failed"; tail "$O/price.err"; exit 1; }
  for a in 1 2; do
    TASX_LIB=$AB TASX_SRV_ACQ=$a timeout -k 10 200 python3 -u tools/price_leg.py "acq$a" >> "$O/price.jsonl" 2>> "$O/price.err" || { echo "price acq$a failed"; tail "$O/price.err"; exit 1; }
  done
  tail -3 "$O/price.jsonl" | cut -c1-500
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o price -- python3 -u tools/price_leg.py traced > "$O/traced.log" 2>&1 || { echo "traced failed"; tail "$O/traced.log"; exit 1; }
tail -1 "$O/traced.log" | cut -c1-500
echo done
