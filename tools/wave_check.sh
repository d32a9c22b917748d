# tcp4_wave_kernel check on the GPU box: parity tests, then the ACK-mix probe
# (tools/ackmix_probe.py) with and without the LDS residency cap.
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${1:-wave}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/ackmix_probe.py --hints ${HINTS:-per} --variants ${VARIANTS:-0,3,8} > $OUT/probe.jsonl 2> $OUT/probe.err || exit $?
[ -n "${BENCH:-}" ] && { timeout -k 10 300 python bench.py --no-pmc > $OUT/bench.log 2>&1 || exit $?; }
echo ok
