# GPU tests + C4 bench line + in-process shard timing (2/4/8 shards, one GPU).
set -o pipefail
OUT=${1:-gpurun_out/q2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench_3.json 2> $OUT/bench_3.err || exit 1
for n in ${SHARDS:-2 4 8}; do
  timeout -k 10 300 python -u tools/shard_bench.py $n 1 > $OUT/bcr_$n.json 2> $OUT/bcr_$n.err || exit 1
done
tail -2 $OUT/tests.log; cat $OUT/bcr_*.json; cut -c1-300 $OUT/bench_3.json
