# round-3 probe: the RX pass with its flow-state key loads non-temporal (A/B
# 43), so that the bucket lines of TAS's flow table can stay in L2 across
# launches: checked bit-exact, timed against the product, read requests counted
set -u
O=gpurun_out/r03r
mkdir -p $O
export TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so TMPDIR=/tmp
timeout -k 10 120 python tools/rx_check.py 43 > $O/check.log 2>&1 || { echo "check failed"; cat $O/check.log; exit 1; }
grep -v amdgpu $O/check.log
for r in 1 2; do for v in 0 43; do
  timeout -k 10 200 python tools/leg_time.py rx --variant $v --reps 2 --tag rx_v$v >> $O/time.jsonl || exit 1
done; done
for v in 0 43; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d "$O/v$v" -o run -- python3 tools/leg_time.py rx --variant $v --steps 16 --reps 1 > "$O/v${v}_pmc.log" 2>&1 || { echo "pmc $v failed"; tail -3 "$O/v${v}_pmc.log"; exit 1; }
done
echo done
