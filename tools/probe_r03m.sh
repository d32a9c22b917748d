# round-3 probe: the fixed host cost of a timed region at the driver's K = 20
# with HSA_ENABLE_INTERRUPT=0 (signal waits by polling) against the default,
# headline leg only, three rounds interleaved
set -u
O=gpurun_out/r03m
mkdir -p $O
for r in 1 2 3; do
  for iv in default 0; do
    if [ $iv = default ]; then
      timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-e2e --no-raw --no-txseg --no-flow --no-flushmix --no-contexts > $O/k20_$iv.r$r.log 2>&1 || { echo "bench failed"; exit 1; }
    else
      HSA_ENABLE_INTERRUPT=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-e2e --no-raw --no-txseg --no-flow --no-flushmix --no-contexts > $O/k20_$iv.r$r.log 2>&1 || { echo "bench failed"; exit 1; }
    fi
    python3 -c "
import json
d=[json.loads(l) for l in open('$O/k20_$iv.r$r.log') if l.startswith('{')][-1]
print(json.dumps({'hsa_enable_interrupt': '$iv', 'round': $r, 'ms_per_step_us': round(d['ms_per_step']*1e3,3), 'launch_avg_us': d['roofline']['launch_avg_us'], 'value': d['value']}))" >> $O/summary.jsonl
  done
done
cat $O/summary.jsonl
