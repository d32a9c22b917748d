set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/txab1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_txseg.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
 for L in tools/bin/ab_HEAD/libtasx.so tas_amd/_lib/libtasx.so; do
  echo "== $L" >> $O/ab.txt
  TASX_LIB=$L timeout -k 10 120 python -u tools/txseg_probe.py --only-kernel --case flows8192_tx16k --steps 200 2>/dev/null | grep -v amdgpu >> $O/ab.txt || exit 1
 done
done
cat $O/ab.txt
