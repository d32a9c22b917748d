set -e
O=gpurun_out/r02p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
echo tests ok
timeout -k 10 300 python -u bench.py --steps 200 > $O/bench.log 2>&1
echo bench ok
