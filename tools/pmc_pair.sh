#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over bench.py's TX segment
# leg (the product, or an A/B variant via TASX_LIB / TASX_TXSEG_DEBUG) and the
# load-scheme probe tools/bin/txseg_lds_probe.  Usage: bash tools/pmc_pair.sh TAG
set -u
TAG=${1:-pair}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
G3="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
i=0
for g in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $g --output-format csv -d "$O/prod_g$i" -o run -- python3 bench.py --pmc-child txseg --steps 16 > "$O/prod_g$i.log" 2>&1 || { echo "prod g$i failed"; exit 1; }
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $g --output-format csv -d "$O/probe_g$i" -o run -- tools/bin/txseg_lds_probe 8 16 > "$O/probe_g$i.log" 2>&1 || { echo "probe g$i failed"; exit 1; }
  echo "group $i done"
done
