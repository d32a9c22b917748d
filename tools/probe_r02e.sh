set -e
mkdir -p gpurun_out/r02e
timeout -k 10 120 python -u tools/sync_overhead.py > gpurun_out/r02e/sync_default.jsonl 2>&1
timeout -k 10 120 python -u tools/sync_overhead.py --spin > gpurun_out/r02e/sync_spin.jsonl 2>&1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02e/ctx -o ctx -- python3 tools/stream_overlap.py --streams 1,2 --steps 100 --rounds 2 > gpurun_out/r02e/ctx.log 2>&1
