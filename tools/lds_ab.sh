# A/B of tcp4_tas14_kernel<NOHINT>'s residency cap on data/ACK mixes and the
# uniform no-hint batch (tools/ackmix_probe.py), interleaved runs.
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${1:-ldsab}; mkdir -p $OUT
for rep in 1 2; do
  for l in 30 0 20; do
    TASX_TAS14_NOHINT_LDS=$l timeout -k 10 200 python tools/ackmix_probe.py --hints none --variants 0 > $OUT/lds${l}_r$rep.jsonl 2>> $OUT/err.log || exit $?
  done
done
echo ok
