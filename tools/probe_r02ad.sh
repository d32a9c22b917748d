set -e
O=gpurun_out/r02ad
mkdir -p $O
for r in 1 2; do
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u tools/ackmix_probe.py --verify --variants 0,9 --hints none --rooms 0,2048 --fracs 0,0.5 > $O/verify_room_r$r.jsonl 2> $O/err.log
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u tools/ackmix_probe.py --verify --offsets --variants 0,9 --hints per,none --rooms 2048 --fracs 0,0.5 > $O/verify_offs_r$r.jsonl 2> $O/err2.log
done
echo done
