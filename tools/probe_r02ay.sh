# TX segment: residency capped by dynamic LDS (3 or 2 blocks per CU) vs the product
set -e
O=gpurun_out/r02ay
mkdir -p $O
TASX_TXSEG_DEBUG=25 TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 300 python -u -m pytest tests/test_txseg.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_dbg25.log 2>&1
echo tests ok
for r in 1 2; do
for d in 0 20 23 24 25; do
TASX_TXSEG_DEBUG=$d TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u bench.py --no-contexts --no-flushmix --no-raw --no-flow --no-e2e --no-cpu-baseline --no-pmc --steps 200 > $O/dbg${d}_r$r.log 2>&1
done
done
echo done
