# bench line after the flow-roofline and two-context changes, at the driver's K=20 and at the default
set -e
O=gpurun_out/r02ba
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/bench_k20.log 2>&1
timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --no-e2e > $O/bench.log 2>&1
echo done
