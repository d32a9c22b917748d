mkdir -p gpurun_out/r05zb
for k in 20 200 20; do
  timeout -k 10 300 python bench.py --steps $k --warmup 5 --no-pmc --no-cpu-baseline --no-server-cost --no-e2e --no-txseg --no-flow --no-contexts --no-flushmix --no-raw > gpurun_out/r05zb/k$k.log 2>&1 || exit 1
  tail -1 gpurun_out/r05zb/k$k.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('K=$k', d['value'], round(d['ms_per_step']*1e3,3), r['launch_avg_us'], r['span_avg_us'], r['frac'], r['read_ceiling']['us'])"
done
