#!/bin/bash
# the headline kernel (tcp4_tas14_kernel<hint>, 65,536
# frames, 98.6 MB algorithmic per launch) against a pure streaming read of the
# same bytes over the same 16 buffers (stream_read_reg_kernel, grid order =
# path 0 and XCD runs of 256 = path 10), counter by counter: where does the
# headline's last few percent to the read ceiling go?  Two --pmc passes per
# kernel form (each within the per-block limits: <= 4 TCC, 4 TCP, 2 TA, 2 GRBM,
# 8 SQ), 8 launches each; the median launch per counter goes to summary.json.
# Usage: bash tools/pmc_read_compare.sh TAG
set -u
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
G1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE TA_TA_BUSY_sum"
G2="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_HIT_sum SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
pass() {  # name group mode [read path]
  local name=$1 g=$2 mode=$3
  TASX_READ_PATH=${4:-0} timeout -k 5 -s KILL 90 rocprofv3 --pmc $g --output-format csv -d "$O/$name" -o run -- \
    python3 bench.py --pmc-child "$mode" --steps 8 > "$O/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$O/$name.log"; exit 1; }
  echo "$name done"
}
i=0
for g in "$G1" "$G2"; do
  i=$((i+1))
  pass head_$i "$g" tcp4
  pass read0_$i "$g" readceil 0
  pass read10_$i "$g" readceil 10
done
python3 - "$O" <<'PY'
import collections, csv, glob, json, sys
o = sys.argv[1]
out = {}
for form, kern in (("head", "tcp4"), ("read0", "stream_read_reg_kernel"),
                   ("read10", "stream_read_reg_kernel")):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{o}/{form}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out[form] = {k: sorted(v)[len(v) // 2] for k, v in sorted(vals.items())}
print(json.dumps(out, indent=1))
json.dump(out, open(f"{o}/summary.json", "w"), indent=1)
PY
