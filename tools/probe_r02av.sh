set -e
O=gpurun_out/r02av
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_c_boundary.py -x -q --timeout 120 --timeout-method thread -m gpu -k "feeder or boundary" > $O/tests.log 2>&1
echo tests ok
for r in 1 2; do
timeout -k 10 200 tools/bin/feeder_bench_ab 3000 7 > $O/two_q7_r$r.jsonl 2> $O/err.log
TASX_FEEDER_ONE_STREAM=1 timeout -k 10 200 tools/bin/feeder_bench_ab 3000 7 > $O/one_q7_r$r.jsonl 2>> $O/err.log
done
echo done
