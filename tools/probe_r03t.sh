# round-3 probe: the shared feeder with 2 (product) or 4 sweeps in flight
# (A/B TASX_FEEDER_SWEEPS=4), 1-8 fast-path threads, 3 and 7 flushes in
# flight per thread (tools/feeder_bench.c built against libtasx_ab.so)
set -u
O=gpurun_out/r03t
mkdir -p $O
for r in 1 2; do
  for sw in 2 4; do
    for q in 3 7; do
      TASX_FEEDER_SWEEPS=$sw timeout -k 10 200 tools/bin/feeder_bench_ab 3000 $q > $O/sw${sw}_q${q}_r$r.jsonl 2>> $O/err.log || { echo "feeder_bench failed"; tail -5 $O/err.log; exit 1; }
    done
  done
done
for f in $O/*.jsonl; do echo "## $f"; cat $f; done
