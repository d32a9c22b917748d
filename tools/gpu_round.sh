#!/bin/bash
# Round-end measurement pass on the GPU box: smoke, GPU tests, the default
# bench line (with PMC traffic), the other BASELINE configs, and the rocprofv3
# kernel-trace summary of the bench.  Each step has its own time limit; a
# crash / timeout / abort ends the script.  Usage: bash tools/gpu_round.sh TAG
set -u
TAG=${1:-r02}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
# a heartbeat: a bench step prints only at its end, which can be minutes
(while sleep 50; do echo "hb $(date +%T)"; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
# PART=a: smoke, GPU tests, the default bench line; PART=b: the rest (one
# gpurun call each; unset: both)
if [ "${PART:-ab}" != "b" ]; then
step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step bench 400 python bench.py
fi
[ "${PART:-ab}" = "a" ] && { echo done; exit 0; }
# the driver's step count: ms_per_step against the event-timed launch
step bench_k20 300 python bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-server-cost
for w in mixed shard8m tso; do
  step bench_$w 300 python bench.py --workload $w --steps 20 --warmup 3
done
# the N>1 code path: bench.py spawns 2 ranks itself; --rehearse lets them
# share this one GPU (gloo control plane; not a scaling measurement)
step bench_n2 300 python bench.py --gpus 2 --rehearse --steps 20 --warmup 3 --no-txseg --no-flow --no-contexts --no-flushmix --no-e2e --no-server-cost
# the RCCL collectives bench.py makes for N > 1, on one rank (RCCL refuses two
# ranks on one GPU; the 8-GPU curve is the driver's run)
step rccl_selftest 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 tools/rccl_selftest.py
export TMPDIR=/tmp
step rocprof_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --no-e2e --no-pmc --no-contexts --no-server-cost --steps 100 --warmup 10
echo done
