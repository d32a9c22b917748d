set -u
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_server.py tests/test_txseg.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | grep -c PASSED; tail -n 25 $O/pytest.log | grep -vE "PASSED"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do timeout -k 10 200 python tools/leg_time.py txseg --reps 2 --tag txseg >> $O/time.jsonl || exit 1; done
python3 -c "
import json
for l in open('$O/time.jsonl'):
    d=json.loads(l); print(d['tag'], d['rep'], d['us'], d['kernel'])"
timeout -k 10 420 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
python3 -c "
import json
for l in open('$O/bench.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); fm=d['e2e']['fastpath_mt']
        print(d['value'], d['roofline']['frac'], d['tx_segment']['cpu_baseline'].get('single_core_us_per_segment'))
        for k,v in fm.items(): print(k, v)"
echo done
