set -e
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "rooms_every_row_mode" --timeout 120 --timeout-method thread > $O/pytest_rows.log 2>&1
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 400 python -u tools/ackmix_probe.py --variants 9,15,16,17,18 --hints per --rooms 0 --fracs 0,0.5,0.75,1 --rounds 2 > $O/ackmix_bs.jsonl
