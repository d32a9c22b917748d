set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
i=0
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d $O/p$i -o run -- python3 tools/txseg_probe.py --only-kernel --case flows8192_tx16k --steps 20 --rotate 4 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
