#!/bin/bash
# Round 5: translation and L2 counters of config 4 (8M x 1500 B RAW, 12.6 GB)
# as bench.py runs it (bench.py --pmc-child shard8m: the product's
# raw_sad_kernel<s32>, XCD runs of 256 blocks), beside the same launches in
# grid order (A/B build, TASX_XRUN=0).  Separate --pmc passes, each within the
# per-block counter limits.  Usage: bash tools/pmc_config4.sh TAG
set -u
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
AB=$PWD/tas_amd/_lib/libtasx_ab.so
P1="TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P2="TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_PENDING_STALL_CYCLES_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TA_TA_BUSY_sum GRBM_UTCL2_BUSY"
i=0
for g in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $g --output-format csv -d "$O/prod$i" -o run -- python3 bench.py --pmc-child shard8m --steps 3 > "$O/prod$i.log" 2>&1 || { echo "prod pass $i failed"; tail -5 "$O/prod$i.log"; exit 1; }
  echo "prod pass $i done"
  TASX_LIB=$AB TASX_XRUN=0 timeout -k 10 -s KILL 150 rocprofv3 --pmc $g --output-format csv -d "$O/grid$i" -o run -- python3 bench.py --pmc-child shard8m --steps 3 > "$O/grid$i.log" 2>&1 || { echo "grid pass $i failed"; tail -5 "$O/grid$i.log"; exit 1; }
  echo "grid pass $i done"
done
python3 - "$O" <<'PY'
import csv, glob, json, sys, collections
o = sys.argv[1]
out = {}
for form in ("prod", "grid"):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{o}/{form}*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "raw_sad_kernel" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out[form] = {k: sorted(v)[len(v) // 2] for k, v in sorted(vals.items())}
print(json.dumps(out, indent=1))
json.dump(out, open(f"{o}/summary.json", "w"), indent=1)
PY
