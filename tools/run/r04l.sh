set -u
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_server.log 2>&1; rc=$?
tail -n 12 $O/pytest_server.log
exit $rc
