set -e
O=gpurun_out/r02n
mkdir -p $O
for r in 1 2; do
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u tools/ackmix_probe.py --variants 9,19 --hints per --rooms 2048 --fracs 0,0.5,1 > $O/f16_r$r.jsonl 2> $O/f16.err
TASX_MIX_F8=1 TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u tools/ackmix_probe.py --variants 19 --hints per --rooms 2048 --fracs 0,0.5,1 > $O/f8_r$r.jsonl 2> $O/f8.err
done
echo done
