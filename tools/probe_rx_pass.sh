# one RX pass (tasx_rx_batch_dev): parity, then the A/B probe against the two calls
set -e
O=gpurun_out/${TAG:-r02bk}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rx_fused.py tests/test_bench_configs.py tests/test_flow.py -x -v -m gpu --timeout 120 --timeout-method thread -k "rx or flow" > $O/tests.log 2>&1
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python tools/rx_probe.py --fracs u,0,0.5,1 --rounds 3 > $O/rx_probe.jsonl 2>&1
echo done
