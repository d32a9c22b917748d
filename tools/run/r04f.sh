set -u
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_server.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_server.log 2>&1 || { echo "server tests failed"; tail -20 $O/pytest_server.log; exit 1; }
tail -n 1 $O/pytest_server.log
fb() { # tag env...
  local tag=$1; shift
  env "$@" TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 1 4 > $O/$tag.q1.jsonl 2>&1 || { echo "$tag q1 failed"; tail -3 $O/$tag.q1.jsonl; exit 1; }
  env "$@" TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 7 4 > $O/$tag.q7.jsonl 2>&1 || { echo "$tag q7 failed"; tail -3 $O/$tag.q7.jsonl; exit 1; }
  grep -h '"mode": "server"' $O/$tag.q1.jsonl $O/$tag.q7.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$tag', d['threads'], d['in_flight'], d['latency_us'], round(d['frames_per_s']/1e6,2))"
  grep -h check $O/$tag.q7.jsonl
}
for r in 1 2; do
  for p in 0 1 2 3 4; do fb fpol${p}_k2_r$r TASX_SRV_K=2 TASX_SRV_FPOL=$p; done
  fb k1_r$r TASX_SRV_K=1
  fb k4_r$r TASX_SRV_K=4
  fb k1_nocold_r$r TASX_SRV_K=1 TASX_SRV_COLD_US=100000000
done
timeout -k 10 300 tools/bin/feeder_bench 3000 7 2 > $O/feeder_q7.jsonl 2>&1 || { echo "feeder failed"; exit 1; }
grep feeder $O/feeder_q7.jsonl
fb vram2 TASX_SRV_VRAM=2 TASX_SRV_K=2
echo done
