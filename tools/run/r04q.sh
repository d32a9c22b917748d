set -u
O=gpurun_out/r04q; mkdir -p $O
AB=$PWD/tas_amd/_lib/libtasx_ab.so
for r in 1 2; do for k in 2 4; do
  TASX_LIB=$AB TASX_SRV_K=$k timeout -k 10 200 python tools/server_k_ab.py --tag k${k}_r$r >> $O/k.jsonl || exit 1
done; done
python3 -c "
import json
for l in open('$O/k.jsonl'):
    d=json.loads(l); print(d['tag'], d['shape'], d['server']['latency_us'], round(d['server']['frames_per_s']/1e6,1), d['txseg_server']['latency_us'], round(d['txseg_server']['segments_per_s']/1e6,2))"
echo done
