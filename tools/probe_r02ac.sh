set -e
O=gpurun_out/r02ac
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
echo tests ok
for r in 1 2; do
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 200 python -u tools/ackmix_probe.py --verify --variants 0,9 --hints per --rooms 0 --fracs 0,0.25,0.5,0.75,1 > $O/verify_r$r.jsonl 2> $O/err.log
done
echo done
