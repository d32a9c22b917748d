# tcp4_wave_kernel check on the GPU box: parity tests, then the ACK-mix probe
# (tools/ackmix_probe.py) with and without the LDS residency cap.
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${1:-wave}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/ackmix_probe.py --hints per > $OUT/probe.jsonl 2> $OUT/probe.err || exit $?
TASX_WAVE_TCP4_LDS=30 timeout -k 10 300 python tools/ackmix_probe.py --hints per --variants 8 > $OUT/probe_lds30.jsonl 2>> $OUT/probe.err || exit $?
echo ok
