# round-3 probe: GPU tests + bench (unless SKIP_ROUND), then A/B variant V (default 37: hint prefetch; 38: row-body fallback) checked bit-exact and timed against the product; output under gpurun_out/$TAG
set -u
O=gpurun_out/${TAG:-r03d}
mkdir -p $O
if [ -z "${SKIP_ROUND:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "tests failed"; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; exit 1; }
fi
export TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so
timeout -k 10 120 python tools/ab_check.py ${V:-37} > $O/ab_check.log 2>&1 || { echo "ab_check failed"; cat $O/ab_check.log; exit 1; }
timeout -k 10 120 python tools/rx_check.py ${V:-37} >> $O/ab_check.log 2>&1 || { echo "rx_check failed"; exit 1; }
for r in 1 2; do for v in 0 ${V:-37}; do for l in flushmix rx_verify rx; do
  timeout -k 10 200 python tools/leg_time.py $l --variant $v --reps 2 --tag ${l}_v$v >> $O/time.jsonl || exit 1
done; done; done
echo done
