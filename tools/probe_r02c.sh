set -e
mkdir -p gpurun_out/r02d
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 300 python -u tools/ackmix_probe.py --variants 9,10,11 --hints per,none --rooms 2048 --fracs 0,0.25,0.5,0.75,1 --rounds 2 > gpurun_out/r02d/ackmix_modes.jsonl
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 300 python -u tools/ackmix_probe.py --offsets --variants 9,10,11 --hints per,none --rooms 2048 --fracs 0,0.5 --rounds 1 > gpurun_out/r02d/ackmix_modes_offs.jsonl
