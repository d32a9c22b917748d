set -u
O=gpurun_out/r04j; mkdir -p $O
export TMPDIR=/tmp
TASX_LIB=$PWD/tas_amd/_lib/libtasx_ab.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/leg_time.py flow --variant 11 --steps 50 --reps 1 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1000,3))"
echo done
