set -u
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_server.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_server.log 2>&1 || { echo "server tests failed"; tail -20 $O/pytest_server.log; exit 1; }
tail -n 1 $O/pytest_server.log
fb() { # tag env...
  local tag=$1; shift
  env "$@" TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 1 4 > $O/$tag.jsonl 2>&1
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$tag rc=$rc"; tail -3 $O/$tag.jsonl; exit 1; fi
  grep -h '"mode": "server' $O/$tag.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if d['threads'] != 1: continue
    if d['mode'] == 'server_diag': print('$tag diag', d['detect_to_loaded_us'], d['loaded_to_acked_us'], d['gap_us'], d['empty_polls_per_batch'])
    else: print('$tag', d['frames_per_flush'], d['latency_us'], d['latency_from_submit_us'], d['core_us_per_flush'])"
}
for r in 1 2; do
  fb prod32_r$r
  fb prod1_r$r FB_BATCH=1
  fb nowork32_r$r TASX_SRV_FPOL=9
  fb nowork1_r$r TASX_SRV_FPOL=9 FB_BATCH=1
  fb sys32_r$r TASX_SRV_FPOL=7
  fb noacq32_r$r TASX_SRV_FPOL=4
  fb vram_nowork32_r$r TASX_SRV_VRAM=2 TASX_SRV_FPOL=9
  fb k1_nowork32_r$r TASX_SRV_K=1 TASX_SRV_FPOL=9
  fb adapt32_r$r TASX_SRV_FPOL=10
done
for r in 1 2; do for p in 0 10; do
  TASX_SRV_FPOL=$p timeout -k 10 200 tools/bin/feeder_bench_ab 3000 3 4 > $O/q3_fpol${p}_r$r.jsonl 2>&1 || { echo "q3 $p failed"; exit 1; }
  grep -h '"mode": "server"' $O/q3_fpol${p}_r$r.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('q3 fpol$p r$r', d['threads'], d['latency_us'], round(d['frames_per_s']/1e6,2))"
done; done
echo done
AB=$PWD/tas_amd/_lib/libtasx_ab.so
timeout -k 10 300 python -u -m pytest tests/test_flow.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_flow.log 2>&1 || { echo "flow tests failed"; tail -20 $O/pytest_flow.log; exit 1; }
tail -n 1 $O/pytest_flow.log
for r in 1 2; do for v in 0 12 13; do
  TASX_LIB=$AB timeout -k 10 200 python tools/leg_time.py flow --variant $v --reps 2 --tag flow_v$v >> $O/time.jsonl || exit 1
done; done
python3 -c "
import json
for l in open('$O/time.jsonl'):
    d=json.loads(l); print(d['tag'], d['rep'], d['us'], d['kernel'])"
for v in 0 12 13; do TASX_LIB=$AB VARIANT=$v PMC_GROUPS="1" bash tools/pmc_legs.sh r04m/pmc flow || exit 1; done
echo done2
