#!/bin/bash
# TX segment build on the GPU box: time the product and A/B variants of
# tx_segment_tas_kernel on bench.py's own tx_segment leg (tools/leg_time.py),
# then PMC passes (one counter group per rocprofv3 run) over the product and
# the no-first-block-write-back ablation (TASX_TXSEG_DEBUG=10), and the
# load-scheme probe tools/bin/txseg_lds_probe.  Usage: bash tools/pmc_txseg.sh TAG [VARIANTS]
set -u
TAG=${1:-txseg}
VARS=${2:-"10"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
AB=$PWD/tas_amd/_lib/libtasx_ab.so
run() { # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
if [ -x tools/bin/txseg_lds_probe ]; then run lds_probe 120 tools/bin/txseg_lds_probe 50; fi
run time_product 120 python3 tools/leg_time.py txseg --tag product
for v in $VARS; do
  TASX_LIB=$AB TASX_TXSEG_DEBUG=$v run time_dbg$v 120 python3 tools/leg_time.py txseg --tag dbg$v
done
G1="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
G2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS"
i=0
for g in "$G1" "$G2"; do
  i=$((i+1))
  run pmc_product_g$i 200 rocprofv3 --pmc $g --output-format csv -d "$O/pmc_product_g$i" -o run -- python3 bench.py --pmc-child txseg --steps 16
  for v in $VARS; do
    TASX_LIB=$AB TASX_TXSEG_DEBUG=$v run pmc_dbg${v}_g$i 200 rocprofv3 --pmc $g --output-format csv -d "$O/pmc_dbg${v}_g$i" -o run -- python3 bench.py --pmc-child txseg --steps 16
  done
done
echo done
