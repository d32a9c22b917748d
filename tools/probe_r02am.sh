set -e
O=gpurun_out/r02am
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
echo tests ok
timeout -k 10 200 tools/bin/feeder_bench 3000 3 > $O/fused_q3.jsonl 2> $O/err.log
timeout -k 10 200 tools/bin/feeder_bench 3000 7 > $O/fused_q7.jsonl 2>> $O/err.log
timeout -k 10 200 tools/bin/flush_bench > $O/flush_bench.jsonl 2>> $O/err.log
echo done
