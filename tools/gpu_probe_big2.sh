#!/bin/bash
# Round 5: XCD-ordered grids across batch sizes (RAW 64K .. 8M x 1500 B; the
# headline's TCP4 frames), chunked XCD runs, allocation order.  Usage: bash tools/gpu_probe_big2.sh TAG
set -eu -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
AB=$PWD/tas_amd/_lib/libtasx_ab.so
timeout -k 10 300 python3 -u tools/big_probe.py --sizes 64,256,1024 --allocs torch --legs prod,v49,v53,v54,v55,v51,read0,read2,read3 > "$O/probe_small.jsonl" 2> "$O/probe.err"
timeout -k 10 300 python3 -u tools/big_probe.py --sizes 8192 --allocs dev,torch --legs prod,v49,v53,v54,v55,v51,read0,read3 > "$O/probe_8m.jsonl" 2>> "$O/probe.err"
for r in 1 2; do
  for v in 0 52 56 57; do
    TASX_LIB=$AB timeout -k 10 120 python3 -u tools/leg_time.py tcp4 --variant $v --steps 400 --reps 2 --tag ab$v >> "$O/headline.jsonl" 2>> "$O/probe.err"
  done
done
echo done
