#!/bin/bash
# bench.py with a heartbeat on stdout (a full bench line takes minutes and
# prints only at its end).  Usage: bash tools/bench_hb.sh OUT.log [bench.py args...]
set -u
out=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p "$(dirname "$out")"
(while sleep 50; do echo "hb $(date +%T)"; done) &
hb=$!
timeout -k 10 500 python bench.py "$@" > "$out" 2>&1
rc=$?
kill $hb
tail -1 "$out" | cut -c1-120
exit $rc
