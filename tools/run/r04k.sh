set -u
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
python3 -c "
import json
for l in open('$O/bench.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); fm=d['e2e']['fastpath_mt']
        print(d['value'], d['roofline']['frac'])
        for k,v in fm.items(): print(k, v)"
echo done
