#!/bin/bash
# TX segment build (bench.py's tx_segment leg) taken apart with the A/B build:
# launch time per TASX_TXSEG_DEBUG variant (tools/leg_time.py), and the
# product on the leg's segments moved so that none wraps.
#   0 product, 30 round-2 product, 31 7 load slots, 32 no fallback compiled in,
#   33 no wraps, 34 both, 35-38 residency capped at 5/4/3/2 blocks per CU
# Usage: bash tools/txseg_split.sh TAG VARIANT...
set -u
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
for v in "$@"; do
  TASX_TXSEG_DEBUG=$v timeout -k 10 200 python tools/leg_time.py txseg --reps 3 --tag d$v >> "$O/time.jsonl" 2>"$O/time_d$v.err" || { echo "time $v failed"; exit 1; }
done
timeout -k 10 200 python tools/leg_time.py txseg_nowrap --reps 3 --tag nowrap_layout >> "$O/time.jsonl" 2>"$O/time_nowrap.err" || { echo "nowrap failed"; exit 1; }
cat "$O/time.jsonl"
