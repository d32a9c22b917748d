set -e
O=gpurun_out/r02k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 tests/c/bin/boundary_test tests/golden/ref_frames.bin > $O/boundary_test.log 2>&1
timeout -k 10 200 tools/bin/flush_bench 200 > $O/flush_bench.jsonl 2> $O/flush_bench.err
