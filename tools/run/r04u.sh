set -u
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_server.log 2>&1; rc=$?
grep -cE "PASSED" $O/pytest_server.log; grep -E "FAILED|ERROR|passed|failed" $O/pytest_server.log | tail -5
exit $rc
