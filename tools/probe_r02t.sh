set -e
O=gpurun_out/r02t
mkdir -p $O
for r in 1 2; do
timeout -k 10 200 tools/bin/flush_bench_ab > $O/frame_starts_r$r.jsonl 2> $O/err.log
TASX_FLUSH_HEADER_RECORDS=1 timeout -k 10 200 tools/bin/flush_bench_ab > $O/header_records_r$r.jsonl 2> $O/err.log
done
echo done
