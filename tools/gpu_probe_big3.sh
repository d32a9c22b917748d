#!/bin/bash
# Round 5: XCD-run lengths (tasx_ab_set_xrun) on config 4's 8M x 1500 B, in
# three processes (three physical layouts), torch and hipMalloc buffers; 256K
# and 1M; configs 3 and 5 with and without XCD runs.  Usage: bash tools/gpu_probe_big3.sh TAG
set -eu -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/$TAG
mkdir -p "$O"
AB=$PWD/tas_amd/_lib/libtasx_ab.so
for r in 1 2 3; do
  timeout -k 10 200 python3 -u tools/big_probe.py --sizes 8192 --allocs torch,dev > "$O/probe_8m_$r.jsonl" 2>> "$O/probe.err"
done
timeout -k 10 200 python3 -u tools/big_probe.py --sizes 256,1024 --allocs torch > "$O/probe_small.jsonl" 2>> "$O/probe.err"
for r in 1 2; do
  for x in 0 9 10; do
    for leg in mixed tso; do
      TASX_XRUN=$x TASX_LIB=$AB timeout -k 10 120 python3 -u tools/leg_time.py $leg --steps 50 --reps 2 --tag x$x >> "$O/legs.jsonl" 2>> "$O/probe.err"
    done
  done
done
echo done
