#!/bin/bash
# The busy flush server's price (bench.py --server-cost-child: the headline and
# the TX build with the server stopped / idle / 8 x 3 busy) per server form
# built by tools/server_variants.py, two alternating rounds, each form in a
# fresh process under TASX_LIB.  Usage: VARS="prod k1" bash tools/server_variants_price.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  for v in ${VARS:-prod k1 notok rows8 rows16 sysld noacq}; do
    TASX_LIB=$PWD/tools/bin/exp_$v/libtasx.so timeout -k 10 200 python bench.py --server-cost-child --rotate 16 > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1])
h=d['headline']; t=d['tx_segment']; f=d['busy_flush_run']
print('$v $r', h['us'], 'headline', h['slowdown_busy'], 'tx', t['slowdown_busy'], 'Mframes/s', round(f['frames_per_s']/1e6,1), 'latency_us', f['latency_us'])"
  done
done
