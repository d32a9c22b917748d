# where the timed region's host time goes at the driver's K=20 (TASX_BENCH_TRACE),
# events created before the timed region
set -e
O=gpurun_out/r02aw2
mkdir -p $O
F="--steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-raw --no-txseg --no-flow --no-flushmix --no-pmc"
for r in 1 2 3; do
TASX_BENCH_TRACE=1 timeout -k 10 300 python bench.py $F > $O/trace_r$r.log 2> $O/trace_r$r.err
done
echo done
