# round-3 probe: A/B 42 (second-generation rows take the other half of the
# first generation's hint lines) checked bit-exact against the product at
# batch sizes around whole generation pairs (TX mix, RX verify, RX pass),
# then timed against it (tools/leg_time.py)
set -u
O=gpurun_out/r03j
mkdir -p $O
export TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so
timeout -k 10 200 python tools/ab_check.py 42 65536,70007,131072,135000 > $O/check.log 2>&1 || { echo "ab_check failed"; cat $O/check.log; exit 1; }
for n in 65536 70007 131072; do
  timeout -k 10 120 python tools/rx_check.py 42 $n >> $O/check.log 2>&1 || { echo "rx_check failed"; cat $O/check.log; exit 1; }
done
grep -v amdgpu $O/check.log
for r in 1 2; do for v in 0 42; do for l in flushmix rx_verify rx; do
  timeout -k 10 200 python tools/leg_time.py $l --variant $v --reps 2 --tag ${l}_v$v >> $O/time.jsonl || exit 1
done; done; done
echo done
