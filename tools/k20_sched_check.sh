#!/bin/bash
# The driver's K = 20 headline line with the host waiting by spinning (bench.py's
# default since round 5) against the runtime's default wait, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05zc
for r in 1 2 3; do
  for sched in spin auto; do
    TASX_BENCH_SCHED=$sched timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-server-cost --no-e2e --no-txseg --no-flow --no-contexts --no-flushmix --no-raw > gpurun_out/r05zc/${sched}_$r.log 2>&1 || exit 1
    tail -1 gpurun_out/r05zc/${sched}_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$sched r$r', d['value'], round(d['ms_per_step']*1e3,3), r['launch_avg_us'], r['span_avg_us'], d['ranks'].get('host_wait'))"
  done
done
