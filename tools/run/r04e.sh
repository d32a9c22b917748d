set -u
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_server.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_server.log 2>&1 || { echo "server tests failed"; tail -20 $O/pytest_server.log; exit 1; }
tail -1 $O/pytest_server.log
for k in 1 8; do
  TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so TASX_SRV_K=$k timeout -k 10 200 python -u -m pytest tests/test_server.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_server_k$k.log 2>&1 || { echo "server tests k$k failed"; tail -20 $O/pytest_server_k$k.log; exit 1; }
  tail -1 $O/pytest_server_k$k.log
done
for r in 1 2; do
  for k in 1 2 4 8; do
    TASX_SRV_K=$k TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 1 4 > $O/srv_q1_k${k}_r$r.jsonl 2>&1 || { echo "fb q1 k$k failed"; tail -3 $O/srv_q1_k${k}_r$r.jsonl; exit 1; }
    TASX_SRV_K=$k TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 7 4 > $O/srv_q7_k${k}_r$r.jsonl 2>&1 || { echo "fb q7 k$k failed"; exit 1; }
  done
  timeout -k 10 300 tools/bin/feeder_bench 3000 7 7 > $O/all_q7_r$r.jsonl 2>&1 || { echo "fb all q7 failed"; exit 1; }
  echo "round $r done"
done
timeout -k 10 120 tools/bin/l2_persist 2 16 > $O/l2_persist.jsonl 2>&1 || { echo "l2_persist failed"; tail -3 $O/l2_persist.jsonl; exit 1; }
cat $O/l2_persist.jsonl
for r in 1 2; do for leg in flow flow_small flow_tiny; do
  timeout -k 10 200 python tools/leg_time.py $leg --reps 2 --tag $leg >> $O/time.jsonl || exit 1
done; done
for v in 0 9; do TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so VARIANT=$v PMC_GROUPS="3" bash tools/pmc_legs.sh r04e/pmc flow || exit 1; done
for vr in 1 2; do
  TASX_SRV_VRAM=$vr TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 1 4 > $O/srv_vram$vr.jsonl 2>&1 || { echo "vram$vr failed"; tail -3 $O/srv_vram$vr.jsonl; exit 1; }
  TASX_SRV_VRAM=$vr TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 7 4 >> $O/srv_vram$vr.jsonl 2>&1 || { echo "vram$vr q7 failed"; exit 1; }
  echo "vram$vr ok"
done
echo done
