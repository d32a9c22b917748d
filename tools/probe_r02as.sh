set -e
O=gpurun_out/r02as
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
echo tests ok
for r in 1 2; do
timeout -k 10 300 python -u bench.py --no-contexts --no-flushmix --no-raw --no-flow --no-e2e --no-cpu-baseline --steps 200 > $O/bench_r$r.log 2>&1
done
echo done
