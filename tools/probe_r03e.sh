# round-3 probe: TX segment A/B 41 (LDS windows by ds_read_b128) checked on the
# TX tests, then the product, the access pattern alone (40), 41 and the
# first block non-temporal (39), interleaved over 3 rounds on one box
set -u
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_txseg.py tests/test_linux_frames.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so
for r in 1 2 3; do for v in 0 40 41 39; do
  TASX_TXSEG_DEBUG=$v timeout -k 10 200 python tools/leg_time.py txseg --reps 2 --tag d$v >> $O/time.jsonl || exit 1
done; done
echo done
