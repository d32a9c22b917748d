set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/wave1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "wave or raw_all_variants or config3 or golden_raw or mixed" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/sweep.py --modes mixed --variants 6,7 --steps 20 --rounds 3 > $O/sweep_main.txt 2>&1 || { tail $O/sweep_main.txt; exit 1; }
cat $O/sweep_main.txt | grep -v amdgpu.ids
for v in wU4 wU8 wL0 wU4L0; do
  TASX_LIB=tools/bin/$v/libtasx.so timeout -k 10 200 python -u tools/sweep.py --modes mixed --variants 7 --steps 20 --rounds 3 > $O/sweep_$v.txt 2>&1 || { tail $O/sweep_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/sweep_$v.txt
done
