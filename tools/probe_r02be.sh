mkdir -p gpurun_out/r02be && timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --no-contexts --no-flushmix --no-raw --no-flow --no-txseg --steps 20 > gpurun_out/r02be/bench.log 2>&1
