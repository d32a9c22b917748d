#!/bin/bash
# Round 5, VERDICT r04 item 1: the config-4 size effect.  Timing legs of
# tools/big_probe.py (product vs trivial read, torch vs hipMalloc buffers, XCD
# order), per-launch drift, the headline with and without the XCD order, and
# three PMC passes over the 8M batch.  Usage: bash tools/gpu_probe_big.sh TAG
set -eu -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
AB=$PWD/tas_amd/_lib/libtasx_ab.so
timeout -k 10 400 python3 -u tools/big_probe.py --sizes ${SIZES:-1,2,8} > "$O/probe.jsonl" 2> "$O/probe.err"
timeout -k 10 120 python3 -u tools/big_probe.py --sizes 8 --allocs torch,dev --sustain 30 > "$O/sustain.jsonl" 2>> "$O/probe.err"
for r in 1 2; do
  for v in 0 52; do
    TASX_LIB=$AB timeout -k 10 120 python3 -u tools/leg_time.py tcp4 --variant $v --steps 400 --reps 3 --tag ab$v >> "$O/headline.jsonl" 2>> "$O/probe.err"
  done
done
P1="TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P2="TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_PENDING_STALL_CYCLES_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TA_TA_BUSY_sum GRBM_UTCL2_BUSY"
P3="TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD"
i=0
for g in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $g --output-format csv -d "$O/pmc$i" -o run -- python3 tools/big_probe.py --pmc > "$O/pmc$i.log" 2>&1
done
echo done
