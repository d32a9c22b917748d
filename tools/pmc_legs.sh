#!/bin/bash
# Read/write request counts by size (one counter group per rocprofv3 run) for
# bench.py legs run by tools/leg_time.py.  Usage: bash tools/pmc_legs.sh TAG LEG...
set -u
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
G1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
G2="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_32B_sum"
for leg in "$@"; do
  i=0
  for g in "$G1" "$G2"; do
    i=$((i+1))
    timeout -k 10 -s KILL 200 rocprofv3 --pmc $g --output-format csv -d "$O/${leg}_g$i" -o run -- python3 tools/leg_time.py $leg --steps 8 --reps 1 > "$O/${leg}_g$i.log" 2>&1 || { echo "$leg g$i failed"; exit 1; }
  done
  echo "$leg done"
done
