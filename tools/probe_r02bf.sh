# fused RX pass: parity first
set -e
O=gpurun_out/r02bf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rx_fused.py tests/test_flow.py tests/test_abi.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo done
