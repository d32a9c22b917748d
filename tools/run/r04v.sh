set -u
O=gpurun_out/r04v; mkdir -p $O
AB=$PWD/tas_amd/_lib/libtasx_ab.so
TASX_LIB=$AB TASX_SRV_FPOL=14 timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -q --timeout 120 --timeout-method thread -k "tx_segments" > $O/pytest_fpol14.log 2>&1
echo "fpol14 tests rc=$?: $(tail -n 1 $O/pytest_fpol14.log)"
for r in 1 2; do for p in 0 14; do
  TASX_LIB=$AB TASX_SRV_FPOL=$p timeout -k 10 200 python tools/server_k_ab.py --tag fpol${p}_r$r >> $O/k.jsonl || exit 1
done; done
python3 -c "
import json
for l in open('$O/k.jsonl'):
    d=json.loads(l); print(d['tag'], d['shape'], d['txseg_server']['latency_us'], round(d['txseg_server']['segments_per_s']/1e6,2))"
echo done
