set -u
O=gpurun_out/r04g; mkdir -p $O
AB=$PWD/tas_amd/_lib/libtasx_ab.so
timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_server.log 2>&1 || { echo "server tests failed"; tail -20 $O/pytest_server.log; exit 1; }
tail -n 1 $O/pytest_server.log
# staleness: the frame-load policies without system scope, on refilled mbufs
for p in 1 2 4 5 6; do
  TASX_LIB=$AB TASX_SRV_FPOL=$p timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -q --timeout 120 --timeout-method thread -k "refilled or reused" > $O/pytest_fpol$p.log 2>&1
  rc=$?; echo "fpol $p rc=$rc: $(tail -n 1 $O/pytest_fpol$p.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping"; exit 1; fi
done
fb() { # tag env...
  local tag=$1; shift
  env "$@" TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 1 4 > $O/$tag.q1.jsonl 2>&1 || { echo "$tag q1 failed"; tail -3 $O/$tag.q1.jsonl; exit 1; }
  env "$@" TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 7 4 > $O/$tag.q7.jsonl 2>&1 || { echo "$tag q7 failed"; tail -3 $O/$tag.q7.jsonl; exit 1; }
  grep -h '"mode": "server"' $O/$tag.q1.jsonl $O/$tag.q7.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$tag', d['threads'], d['in_flight'], d['latency_us'], round(d['frames_per_s']/1e6,2))"
}
for r in 1 2; do
  for k in 2 4; do for p in 0 4 5 6; do fb fpol${p}_k${k}_r$r TASX_SRV_K=$k TASX_SRV_FPOL=$p; done; done
  for p in 0 4 5; do fb malloc_fpol${p}_k2_r$r FB_MALLOC=1 TASX_SRV_K=2 TASX_SRV_FPOL=$p; done
done
timeout -k 10 300 tools/bin/feeder_bench 3000 7 2 > $O/feeder_q7.jsonl 2>&1 || { echo "feeder failed"; exit 1; }
grep feeder $O/feeder_q7.jsonl
FB_MALLOC=1 timeout -k 10 300 tools/bin/feeder_bench 3000 7 2 > $O/feeder_malloc_q7.jsonl 2>&1 || { echo "feeder malloc failed"; exit 1; }
grep feeder $O/feeder_malloc_q7.jsonl
echo done
