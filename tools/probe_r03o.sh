# round-3 probe: the TX segment leg's box-to-box spread -- the product and its
# access pattern alone (A/B 40), interleaved, beside the device's streaming
# copy of the same bytes (bench.copy_ceiling), on whatever box this call gets
set -u
O=gpurun_out/r03o_${1:-a}
mkdir -p $O
export TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so
for r in 1 2; do for v in 0 40; do
  TASX_TXSEG_DEBUG=$v timeout -k 10 200 python tools/leg_time.py txseg --reps 2 --tag d$v >> $O/time.jsonl || exit 1
done; done
timeout -k 10 120 python -c "
import json, bench, torch
from tas_amd import xsum
xsum.lib()
tw = bench.TxSegWorkload(2, 1)
print(json.dumps({'copy_ceiling': bench.copy_ceiling(int(tw.block_floor['bytes']) // 2)}))" >> $O/time.jsonl 2>/dev/null || exit 1
cat $O/time.jsonl
