set -e
O=gpurun_out/r02g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 60 tools/bin/fetch_calib > $O/fetch_calib.jsonl
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fc1 -o fc -- tools/bin/fetch_calib > /dev/null 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/fc2 -o fc -- tools/bin/fetch_calib > /dev/null 2>&1 || echo "pass2 failed"
timeout -k 10 120 tools/bin/flow_ceiling 200 > $O/flow_ceiling.jsonl 2>&1
