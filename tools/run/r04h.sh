set -u
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_server.log 2>&1 || { echo "server tests failed"; tail -20 $O/pytest_server.log; exit 1; }
tail -n 1 $O/pytest_server.log
for r in 1 2; do
  timeout -k 10 300 tools/bin/feeder_bench 3000 1 7 > $O/all_q1_r$r.jsonl 2>&1 || { echo "fb q1 failed"; tail -3 $O/all_q1_r$r.jsonl; exit 1; }
  timeout -k 10 300 tools/bin/feeder_bench 3000 3 6 > $O/fs_q3_r$r.jsonl 2>&1 || { echo "fb q3 failed"; exit 1; }
  timeout -k 10 300 tools/bin/feeder_bench 3000 7 6 > $O/fs_q7_r$r.jsonl 2>&1 || { echo "fb q7 failed"; exit 1; }
  FB_MALLOC=1 timeout -k 10 300 tools/bin/feeder_bench 3000 7 4 > $O/srv_malloc_q7_r$r.jsonl 2>&1 || { echo "fb malloc failed"; exit 1; }
  cat $O/all_q1_r$r.jsonl $O/fs_q3_r$r.jsonl $O/fs_q7_r$r.jsonl $O/srv_malloc_q7_r$r.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if 'threads' in d: print('r$r', d['mode'], d['threads'], d['in_flight'], d['latency_us'], round(d['frames_per_s']/1e6,2), d['core_us_per_flush'])
    elif 'check' in d: print(d)"
done
echo done
