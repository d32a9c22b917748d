# A/B of the no-hint RX verification kernel (tcp4_tas14_kernel<VERIFY, NOHINT>)
# on data/ACK mixes: register budget (TASX_TAS14_WPE) x LDS residency cap
# (TASX_TAS14_VERIFY_LDS, KiB), after the GPU parity tests.
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${1:-verifyab}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for cfg in "6 30" "8 30" "8 0"; do
    set -- $cfg
    TASX_TAS14_WPE=$1 TASX_TAS14_VERIFY_LDS=$2 timeout -k 10 200 python tools/ackmix_probe.py --verify --hints per --variants 0 --fracs 0,0.25,0.5,0.75 > $OUT/w$1_l$2_r$rep.jsonl 2>> $OUT/err.log || exit $?
  done
done
echo ok
