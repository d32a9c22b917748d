#!/bin/bash
# The bench line's e2e fast-path legs (tasxb_fastpath_mt: per-context, feeder,
# server, TX segments through the server at 1 x 1, 8 x 3, 8 x 7) and its
# server_cost leg per server form built by tools/server_variants.py, two
# alternating rounds.  Usage: VARS="prod k1" bash tools/server_variants_e2e.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; mkdir -p $O
for r in 1 2; do
  for v in ${VARS:-prod k1 notok}; do
    TASX_LIB=$PWD/tools/bin/exp_$v/libtasx.so timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --no-raw --no-txseg --no-flow --no-config4 --no-flushmix --no-contexts --steps 50 --warmup 5 > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1])
f=d['e2e']['fastpath_mt']; s=d['server_cost']
print('$v $r', 'headline', s['headline']['slowdown_busy'], 'tx', s['tx_segment']['slowdown_busy'], 'meanwhile', s['busy_flush_run']['frames_per_s_meanwhile'])
for k in ('server_1x1', 'server_8x3', 'server_8x7', 'txseg_server_1x1', 'txseg_server_8x3', 'txseg_server_8x7'):
    print('   ', k, f[k])
print('    flush32_server_us', d['e2e']['flush32_server_us'])"
  done
done
