set -e
O=gpurun_out/r02aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rooms_every_row_mode or flush_mix" > $O/tests.log 2>&1
echo tests ok
for r in 1 2 3; do
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u tools/ackmix_probe.py --variants 20,21 --hints per --rooms 2048 --fracs 0,0.25,0.5,0.75,1 > $O/ackmix_r$r.jsonl 2> $O/ackmix.err
done
echo done
