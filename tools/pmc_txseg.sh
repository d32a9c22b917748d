#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over the fused TX segment
# build and, for comparison, the copy probe (tools/bin/copy_unaligned).
# Usage on the GPU box: bash tools/pmc_txseg.sh   (results under gpurun_out/pmc)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc
mkdir -p $O
i=0
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAVES" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/k$i -o run -- python3 tools/txseg_probe.py --only-kernel --case flows8192_tx16k --steps 20 --rotate 4 > $O/k$i.log 2>&1
  rc=$?; echo "kernel pass $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/c$i -o run -- tools/bin/copy_unaligned 4 10 > $O/c$i.log 2>&1
  rc=$?; echo "copy pass $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
