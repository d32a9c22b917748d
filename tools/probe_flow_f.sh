# flow lookup with F frames per lane: parity, then the A/B probe and the RX pass
set -e
O=gpurun_out/${TAG:-r02cb}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_flow.py tests/test_rx_fused.py tests/test_bench_configs.py -x -v -m gpu --timeout 120 --timeout-method thread -k "flow or rx" > $O/tests.log 2>&1
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python tools/flow_probe.py --variants 1,6,8,7 --rounds 5 > $O/flow_probe.jsonl 2>&1
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python tools/rx_probe.py --fracs u,0,0.5,1 --rounds 2 > $O/rx_probe.jsonl 2>&1
echo done
