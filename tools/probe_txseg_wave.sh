# one-segment-per-wave TX segment build (A/B TASX_TXSEG_DEBUG=29): parity on
# every TX segment case, then the bench leg against the product, twice each
set -e
O=gpurun_out/${TAG:-r02bq}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_txseg.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  for v in 0 29; do
    TASX_LIB=tas_amd/_lib/libtasx_ab.so TASX_TXSEG_DEBUG=$v timeout -k 10 200 python bench.py --no-pmc --no-cpu-baseline --no-e2e --no-raw --no-flow --no-flushmix --no-contexts --steps 200 > $O/bench_$v.r$r.log 2>&1
  done
done
echo done
