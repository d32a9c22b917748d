set -e
O=gpurun_out/r02q
mkdir -p $O
for r in 1 2; do
for lds in 0 10 20 30; do
TASX_TAS14_NOHINT_LDS=$lds TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u tools/ackmix_probe.py --variants 0 --hints per --rooms 2048 --fracs 0,0.5,1 > $O/lds${lds}_r$r.jsonl 2> $O/err.log
done
done
echo done
