set -e
O=gpurun_out/r02ar
mkdir -p $O
TASX_TXSEG_DEBUG=19 TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 300 python -u -m pytest tests/test_txseg.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_dbg19.log 2>&1
echo tests ok
for r in 1 2; do
for d in 0 16 19; do
TASX_TXSEG_DEBUG=$d TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u bench.py --no-contexts --no-flushmix --no-raw --no-flow --no-e2e --no-cpu-baseline --steps 200 > $O/dbg${d}_r$r.log 2>&1
echo "dbg $d r $r"
done
done
