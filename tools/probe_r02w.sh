set -e
O=gpurun_out/r02w
mkdir -p $O
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM"
timeout -s KILL 240 rocprofv3 --pmc $C -d $O/txseg --output-format csv -- python3 bench.py --no-contexts --no-flushmix --no-flow --no-e2e --no-cpu-baseline --no-pmc --no-raw --steps 20 --warmup 3 > $O/txseg.log 2>&1
echo txseg
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/copy --output-format csv -- tools/bin/copy_unaligned 8 10 > $O/copy.log 2>&1
echo copy
