#!/bin/bash
# RX pass (bench.py's rx_pass leg, 64K frames, half ACKs) taken apart with the
# A/B build: each variant's launch time (tools/leg_time.py) and its L2 -> memory
# side read requests by size (one counter group per rocprofv3 run), and the
# XCD-matched split grid checked bit-exact against the product
# (tools/rx_check.py).  Usage: bash tools/rx_split.sh TAG VARIANT...
#   0 product (since r03c: lookup blocks on their verify blocks' XCD, then
#   A/B 32; 36 = the round-2 product), 28 lookup blocks
#   after their verify blocks, 29 no frame key load, 31 no flow-state key load,
#   33 no bucket loads, 34 the frame key only
set -u
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
for v in 36 28; do
  timeout -k 10 120 python tools/rx_check.py $v >> "$O/check.log" 2>&1 || { echo "check $v failed"; exit 1; }
done
cat "$O/check.log"
for v in "$@"; do
  timeout -k 10 200 python tools/leg_time.py rx --variant $v --reps 3 --tag v$v >> "$O/time.jsonl" 2>"$O/time_v$v.err" || { echo "time $v failed"; exit 1; }
done
cat "$O/time.jsonl"
G1="FETCH_SIZE"
G2="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
for v in "$@"; do
  i=0
  for g in "$G1" "$G2"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$O/v${v}_g$i" -o run -- python3 tools/leg_time.py rx --variant $v --steps 8 --reps 1 > "$O/v${v}_g$i.log" 2>&1 || { echo "pmc $v g$i failed"; exit 1; }
  done
  echo "pmc $v done"
done
