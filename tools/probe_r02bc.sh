# TX segment build from pinned host memory: hipHostMalloc default vs coherent vs non-coherent (A/B)
set -e
O=gpurun_out/r02bc
mkdir -p $O
F="--no-pmc --no-cpu-baseline --no-contexts --no-flushmix --no-raw --no-flow --no-txseg --steps 20"
for r in 1 2; do
for fl in 0 0x40000000 0x80000000; do
TASX_HOST_ALLOC_FLAGS=$fl TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 300 python -u bench.py $F > $O/bench_$fl.r$r.log 2>&1
done
done
TASX_HOST_ALLOC_FLAGS=0x80000000 TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 300 python -u -m pytest tests/test_txseg.py -x -q -m gpu --timeout 120 --timeout-method thread -k "host_memory" > $O/tests_nc.log 2>&1
echo done
