#!/bin/bash
# The driver's K = 20 headline line with the timed region's host phases
# printed (TASX_BENCH_TRACE=1: start record, issue of the K launches, end
# record, the final synchronize; event span), 3 runs.
O=gpurun_out/${1:-r05k20t}
mkdir -p $O
for r in 1 2 3; do
  TASX_BENCH_TRACE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-server-cost --no-e2e --no-txseg --no-flow --no-contexts --no-flushmix --no-raw > $O/k20_$r.log 2> $O/k20_$r.err || exit 1
  grep '"K": 20' $O/k20_$r.err | tail -3
  tail -1 $O/k20_$r.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('run $r', d['value'], round(d['ms_per_step']*1e3,3), r['launch_avg_us'], r['span_avg_us'])"
done
