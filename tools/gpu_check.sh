#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash / timeout / abort ends the
# script (rc not in {0,1}); a plain test failure (rc 1) still lets the
# measurement run.  Usage: bash tools/gpu_check.sh [tag] [bench args...]
set -u
TAG=${1:-r01}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step bench 300 python bench.py "$@"
export TMPDIR=/tmp
step rocprof_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --no-e2e --no-pmc --no-contexts --no-flushmix --steps 100 --warmup 10
echo done
