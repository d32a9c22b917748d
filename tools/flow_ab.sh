# flow lookup A/B on the GPU box: parity tests, then the variants interleaved,
# then the no-CRC diagnostic build (what the hash costs on the dependent chain)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/flow1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_flow.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/flow_probe.py --variants 1,3,5 --rounds 5 > $O/probe.txt 2>&1 || { tail $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
TASX_LIB=tools/bin/fnocrc/libtasx.so timeout -k 10 300 python -u tools/flow_probe.py --variants 1,5 --rounds 5 --no-check > $O/probe_nocrc.txt 2>&1 || { tail $O/probe_nocrc.txt; exit 1; }
echo "== no-CRC diag build (variant 5 = no hash)"; grep -v amdgpu.ids $O/probe_nocrc.txt
