# TX segment build from pinned host memory: parity, then the e2e bench leg
set -e
O=gpurun_out/r02bb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_txseg.py -x -v -m gpu --timeout 120 --timeout-method thread -k "host_memory" > $O/tests.log 2>&1
echo tests ok
timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --no-contexts --no-flushmix --no-raw --no-flow --no-txseg --steps 20 > $O/bench.log 2>&1
echo done
