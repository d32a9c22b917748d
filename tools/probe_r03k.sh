# round-3 probe: why the TX segment build's time varies from box to box --
# translation (UTCL1) and memory-side stall counters of the TX leg beside the
# headline leg, one counter group per rocprofv3 run, and the leg's time on the box
set -u
O=gpurun_out/r03k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/leg_time.py txseg --reps 3 --tag txseg > $O/time.jsonl 2>/dev/null || exit 1
G1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum"
G2="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum"
G3="GRBM_UTCL2_BUSY GRBM_TA_BUSY"
for leg in txseg tcp4; do
  i=0
  for g in "$G1" "$G2" "$G3"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$O/${leg}_g$i" -o run -- python3 tools/leg_time.py $leg --steps 8 --reps 1 > "$O/${leg}_g$i.log" 2>&1 || { echo "$leg g$i failed"; tail -3 "$O/${leg}_g$i.log"; exit 1; }
  done
done
cat $O/time.jsonl
echo done
