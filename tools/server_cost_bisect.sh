mkdir -p gpurun_out/r05q
B="--no-cpu-baseline --no-pmc --no-e2e"
i=0
for extra in "" "--no-flow" "--no-contexts --no-flushmix" "--no-txseg --no-raw"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $B $extra > gpurun_out/r05q/b$i.log 2>&1 || { echo "bench $i failed"; tail -5 gpurun_out/r05q/b$i.log; exit 1; }
  echo "b$i [$extra] done"
done
