set -e
O=gpurun_out/r02m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "mix_kernel or rooms_every_row_mode or selects_row_mode" > $O/tests.log 2>&1
echo tests ok
TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 300 python -u tools/ackmix_probe.py --variants 9,19 --hints per --rooms 2048 --fracs 0,0.25,0.5,0.75,1 --rounds 2 > $O/ackmix.jsonl 2> $O/ackmix.err
echo probe ok
timeout -k 10 200 python -u bench.py --no-contexts --no-raw --no-txseg --no-flow --no-e2e --no-cpu-baseline --no-pmc --steps 200 > $O/bench.log 2>&1
echo bench ok
