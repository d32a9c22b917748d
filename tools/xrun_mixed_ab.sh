#!/bin/bash
# Config 3 (1M mixed-MTU RAW, raw_wave_kernel, 65,536 blocks) with the XCD run
# length swept (A/B build, TASX_XRUN: 7/8/9/10 = runs of 64/128/256/512; the
# product uses 9), two alternating rounds.  Usage: bash tools/xrun_mixed_ab.sh TAG
set -u
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
AB=$PWD/tas_amd/_lib/libtasx_ab.so
for r in 1 2; do
  for x in 7 8 9 10; do
    TASX_LIB=$AB TASX_XRUN=$x timeout -k 10 200 python bench.py --workload mixed --steps 50 --warmup 5 --no-pmc --no-cpu-baseline > "$O/x${x}_r$r.log" 2>&1 || { echo "x$x failed"; tail -5 "$O/x${x}_r$r.log"; exit 1; }
    tail -1 "$O/x${x}_r$r.log" | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('x$x r$r', r['launch_avg_us'], r['frac'], r['read_ceiling']['us'])"
  done
done
