set -e
O=gpurun_out/r02l
mkdir -p $O
for r in 1 2; do
for lds in 0 20 30 40 54 80; do
  TASX_LIB=tas_amd/_lib/libtasx_ab.so TASX_TAS14_HINT_LDS=$lds timeout -k 10 120 python -u bench.py --no-contexts --no-flushmix --no-raw --no-txseg --no-flow --no-e2e --no-cpu-baseline --no-pmc --steps 200 > $O/lds${lds}_r$r.log 2>&1
  echo "lds $lds r $r done"
done
done
