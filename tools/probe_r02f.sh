set -e
mkdir -p gpurun_out/r02f
timeout -k 10 120 tools/bin/flow_ceiling 200 > gpurun_out/r02f/flow_ceiling.jsonl 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02f/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --no-pmc > gpurun_out/r02f/bench.log 2>&1
