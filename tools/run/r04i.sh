set -u
O=gpurun_out/r04i; mkdir -p $O
AB=$PWD/tas_amd/_lib/libtasx_ab.so
timeout -k 10 300 python -u -m pytest tests/test_flow.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_flow.log 2>&1 || { echo "flow tests failed"; tail -20 $O/pytest_flow.log; exit 1; }
tail -n 1 $O/pytest_flow.log
for r in 1 2 3; do for v in 0 11; do
  TASX_LIB=$AB timeout -k 10 200 python tools/leg_time.py flow --variant $v --reps 2 --tag flow_v$v >> $O/time.jsonl || exit 1
done; done
python3 -c "
import json
for l in open('$O/time.jsonl'):
    d=json.loads(l); print(d['tag'], d['rep'], d['us'], d['kernel'])"
TASX_LIB=$AB VARIANT=11 PMC_GROUPS="3" bash tools/pmc_legs.sh r04i/pmc flow || exit 1
echo done
