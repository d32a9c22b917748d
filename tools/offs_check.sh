# tcp4_tas14_kernel<OFFS> check on the GPU box: parity tests, then the ACK-mix
# probe in offsets mode (automatic = tcp4_tas14_kernel<OFFS>, 2 = tcp4_frame_kernel).
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${1:-offs}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ackmix_probe.py --offsets --hints none,per --variants 0,2 > $OUT/probe.jsonl 2> $OUT/probe.err || exit $?
echo ok
