set -u
O=gpurun_out/r04n; mkdir -p $O
AB=$PWD/tas_amd/_lib/libtasx_ab.so
timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_server.log 2>&1 || { echo "server tests failed"; tail -30 $O/pytest_server.log; exit 1; }
tail -n 1 $O/pytest_server.log
TASX_LIB=$AB TASX_SRV_FPOL=11 timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -q --timeout 120 --timeout-method thread -k "refilled or reused" > $O/pytest_fpol11.log 2>&1
echo "fpol 11 staleness rc=$?: $(tail -n 1 $O/pytest_fpol11.log)"
for r in 1 2 3; do for p in 0 11; do
  TASX_SRV_FPOL=$p TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 1 4 > $O/q1_fpol${p}_r$r.jsonl 2>&1 || { echo "q1 $p failed"; exit 1; }
  TASX_SRV_FPOL=$p timeout -k 10 200 tools/bin/feeder_bench_ab 3000 3 4 > $O/q3_fpol${p}_r$r.jsonl 2>&1 || { echo "q3 $p failed"; exit 1; }
  cat $O/q1_fpol${p}_r$r.jsonl $O/q3_fpol${p}_r$r.jsonl | grep '"mode": "server"' | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('fpol$p r$r', d['threads'], d['in_flight'], d['latency_us'], round(d['frames_per_s']/1e6,2))"
done; done
echo done
