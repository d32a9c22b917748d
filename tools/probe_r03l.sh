# round-3 probe: the fixed host cost of a timed region at the driver's K = 20
# with and without HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device
# memory), headline leg only, three runs each, interleaved
set -u
O=gpurun_out/r03l
mkdir -p $O
for r in 1 2 3; do
  for kv in 0 1; do
    HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-e2e --no-raw --no-txseg --no-flow --no-flushmix --no-contexts > $O/k20_kv${kv}_r$r.log 2>&1 || { echo "bench failed"; exit 1; }
    python3 -c "
import json,sys
d=[json.loads(l) for l in open('$O/k20_kv${kv}_r$r.log') if l.startswith('{')][-1]
print(json.dumps({'kernarg_dev': $kv, 'round': $r, 'ms_per_step_us': round(d['ms_per_step']*1e3,3), 'launch_avg_us': d['roofline']['launch_avg_us'], 'value': d['value']}))" >> $O/summary.jsonl
  done
done
cat $O/summary.jsonl
