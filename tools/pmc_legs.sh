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
# L2 hit / miss beside the memory-side requests (round 4: where the flow tables' lines are served)
G3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
# PMC_GROUPS="1 2 3" (default "1 2"); VARIANT=v runs tools/leg_time.py --variant v (A/B variants need TASX_LIB)
for leg in "$@"; do
  for gi in ${PMC_GROUPS:-1 2}; do
    g=$(eval echo \$G$gi)
    d="$O/${leg}_v${VARIANT:-0}_g$gi"
    timeout -k 10 -s KILL 200 rocprofv3 --pmc $g --output-format csv -d "$d" -o run -- python3 tools/leg_time.py $leg --variant ${VARIANT:-0} --steps 8 --reps 1 > "$d.log" 2>&1 || { echo "$leg g$gi failed"; exit 1; }
  done
  echo "$leg done"
done
