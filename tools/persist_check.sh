# persistent flush kernel on the GPU box: its parity test (time-limited), then
# the C flush-latency bench with the persistent column
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/persist; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 60 --timeout-method thread -k "persistent or zero_copy or deferred" > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/bin/flush_bench 200 > $O/flush.jsonl 2> $O/flush.err
rc=$?; cat $O/flush.jsonl $O/flush.err; exit $rc
