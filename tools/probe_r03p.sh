# round-3 probe: the no-hint forms (whole-room rows, total_length-first rows)
# with the headline's residency (A/B 43 / 44) checked bit-exact and timed
# against the product's 8-waves-per-SIMD rows
set -u
O=gpurun_out/r03p
mkdir -p $O
export TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so
for v in 43 44; do
  timeout -k 10 120 python tools/nohint_check.py $v >> $O/check.log 2>&1 || { echo "check $v failed"; cat $O/check.log; exit 1; }
done
grep -v amdgpu $O/check.log
for r in 1 2; do
  for v in 0 43; do timeout -k 10 200 python tools/leg_time.py tcp4_nohint --variant $v --reps 2 --tag nohint_v$v >> $O/time.jsonl || exit 1; done
  for v in 0 44; do timeout -k 10 200 python tools/leg_time.py tcp4_frames_only --variant $v --reps 2 --tag frames_only_v$v >> $O/time.jsonl || exit 1; done
done
echo done
