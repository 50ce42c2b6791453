# Sharded-path check on one GPU: sharded parity tests (both reduced solvers),
# then the in-process shard timing (tools/shard_bench.py) for 2 and 4 shards
# with the all-reduced BCR and with the partitioned chain.
set -o pipefail
OUT=${1:-gpurun_out/shard}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
for n in 2 4; do
  timeout -k 10 200 python -u tools/shard_bench.py $n 2 > $OUT/bcr_$n.json 2> $OUT/bcr_$n.err || exit 1
  MMBA_SHARD_BCR=0 timeout -k 10 200 python -u tools/shard_bench.py $n 2 > $OUT/part_$n.json 2> $OUT/part_$n.err || exit 1
done
cat $OUT/*.json
