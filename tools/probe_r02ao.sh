set -e
O=gpurun_out/r02ao
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rooms_every_row_mode" > $O/tests.log 2>&1
echo tests ok
for r in 1 2; do
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u tools/ackmix_probe.py --variants 20,22,23,24,25 --hints per --rooms 2048 --fracs 0.5 > $O/bs_r$r.jsonl 2> $O/err.log
done
echo done
