# A/B of tcp4_tas14_kernel<NOHINT> register budgets (TASX_TAS14_WPE = waves per
# SIMD the compiler must allow; unset = 74 VGPRs, 6 waves) on data/ACK mixes.
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${1:-wpeab}; mkdir -p $OUT
for rep in 1 2; do
  for w in 6 7 8; do
    TASX_TAS14_WPE=$w timeout -k 10 200 python tools/ackmix_probe.py --hints none --variants 0 --fracs 0,0.25,0.5,0.75,1 > $OUT/wpe${w}_r$rep.jsonl 2>> $OUT/err.log || exit $?
  done
done
echo ok
