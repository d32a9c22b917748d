set -u
O=gpurun_out/r04d; mkdir -p $O
export TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so
for pm in 0 1 2 3; do
  TASX_SRV_POLL=$pm timeout -k 10 200 python -u -m pytest tests/test_server.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_server_pm$pm.log 2>&1 || { echo "server tests pm$pm failed"; tail -20 $O/pytest_server_pm$pm.log; exit 1; }
  tail -1 $O/pytest_server_pm$pm.log
done
for r in 1 2; do for pm in 0 1 2 3; do
  TASX_SRV_POLL=$pm TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 1 4 > $O/srv_diag_q1_pm${pm}_r$r.jsonl 2>&1 || { echo "fb q1 failed"; tail -3 $O/srv_diag_q1_pm${pm}_r$r.jsonl; exit 1; }
  TASX_SRV_POLL=$pm TASX_SRV_DIAG=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 7 4 > $O/srv_diag_q7_pm${pm}_r$r.jsonl 2>&1 || { echo "fb q7 failed"; exit 1; }
done; done
timeout -k 10 300 tools/bin/feeder_bench_ab 3000 7 2 > $O/feeder_q7.jsonl 2>&1 || { echo "feeder q7 failed"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_txseg.py tests/test_gpu_parity.py tests/test_flow.py -k "ldsdma or lane_groups or txseg or flow" -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for v in 0 44 40; do
  TASX_TXSEG_DEBUG=$v timeout -k 10 200 python tools/leg_time.py txseg --reps 2 --tag tx_d$v >> $O/time.jsonl || exit 1
done; done
for r in 1 2; do for v in 0 45 46 47 48; do
  timeout -k 10 200 python tools/leg_time.py raw --variant $v --reps 2 --tag raw_v$v >> $O/time.jsonl || exit 1
  timeout -k 10 200 python tools/leg_time.py shard1m --variant $v --steps 40 --reps 2 --tag shard1m_v$v >> $O/time.jsonl || exit 1
done; done
for v in 0 45 46 47; do
  timeout -k 10 200 python tools/leg_time.py shard8m --variant $v --steps 6 --reps 2 --tag shard8m_v$v >> $O/time.jsonl || exit 1
done
for r in 1 2; do for v in 0 9 10; do
  timeout -k 10 200 python tools/leg_time.py flow --variant $v --reps 2 --tag flow_v$v >> $O/time.jsonl || exit 1
done; done
for v in 0 9 10; do VARIANT=$v GROUPS="3" bash tools/pmc_legs.sh r04d/pmc flow || exit 1; done
echo done
