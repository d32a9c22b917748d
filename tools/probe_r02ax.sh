# TX segment: DPP tail (no ds_bpermute round trips) and occupancy 5 (WPE 5) vs the product
set -e
O=gpurun_out/r02ax
mkdir -p $O
for d in 20 21 22; do
TASX_TXSEG_DEBUG=$d TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 300 python -u -m pytest tests/test_txseg.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_dbg$d.log 2>&1
done
echo tests ok
for r in 1 2; do
for d in 0 20 21 22; do
TASX_TXSEG_DEBUG=$d TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u bench.py --no-contexts --no-flushmix --no-raw --no-flow --no-e2e --no-cpu-baseline --no-pmc --steps 200 > $O/dbg${d}_r$r.log 2>&1
done
done
echo done
