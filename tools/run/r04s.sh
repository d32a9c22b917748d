set -u
O=gpurun_out/r04s; mkdir -p $O
AB=$PWD/tas_amd/_lib/libtasx_ab.so
for r in 1 2; do for p in 0 12; do
  TASX_LIB=$AB TASX_SRV_FPOL=$p timeout -k 10 200 python tools/server_k_ab.py --tag fpol${p}_r$r >> $O/k.jsonl || exit 1
done; done
python3 -c "
import json
for l in open('$O/k.jsonl'):
    d=json.loads(l); print(d['tag'], d['shape'], d['txseg_server']['latency_us'], round(d['txseg_server']['segments_per_s']/1e6,2))"
echo done
