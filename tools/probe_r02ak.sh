set -e
O=gpurun_out/r02ak
mkdir -p $O
TASX_POST_WRITEVALUE=1 TASX_LIB=tas_amd/_lib/libtasx_ab.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "flush or feeder or zero_copy" > $O/tests_wv.log 2>&1
echo tests ok
for r in 1 2; do
timeout -k 10 200 tools/bin/feeder_bench_ab 3000 3 > $O/kernel_q3_r$r.jsonl 2> $O/err.log
TASX_POST_WRITEVALUE=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 3 > $O/wv_q3_r$r.jsonl 2>> $O/err.log
done
echo done
