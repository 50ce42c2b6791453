# Sharded-path GPU cycle: sharded parity/structure tests (2-8 shards, in-process
# transport), then the full-size weak-scaling scene at 2, 4 and 8 shards on one GPU.
set -o pipefail
OUT=${1:-gpurun_out/shard}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed" >> $OUT/tests.log; tail -30 $OUT/tests.log; exit 1; }
for n in 2 4 8; do
  timeout -k 10 300 python -u tools/shard_bench.py $n 1 > $OUT/shard_$n.json 2> $OUT/shard_$n.err || exit 1
done
echo "all done"
