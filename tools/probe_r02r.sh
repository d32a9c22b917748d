set -e
O=gpurun_out/r02r
mkdir -p $O
for r in 1 2; do
for d in 0 7 8; do
TASX_TXSEG_DEBUG=$d TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u bench.py --no-contexts --no-flushmix --no-raw --no-flow --no-e2e --no-cpu-baseline --no-pmc --steps 200 > $O/dbg${d}_r$r.log 2>&1
echo "dbg $d r $r"
done
done
