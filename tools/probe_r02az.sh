# TX segment: where the product's time goes beyond the bare load/store pattern
# (timing-only ablations 26-28; 10 = the round-1 no-write-back ablation)
set -e
O=gpurun_out/r02az
mkdir -p $O
for r in 1 2; do
for d in 0 10 26 27 28; do
TASX_TXSEG_DEBUG=$d TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u bench.py --no-contexts --no-flushmix --no-raw --no-flow --no-e2e --no-cpu-baseline --no-pmc --steps 200 > $O/dbg${d}_r$r.log 2>&1
done
done
echo done
