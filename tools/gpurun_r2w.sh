# BCR dataflow phase probe + the relaxed sharded test
set -o pipefail
OUT=gpurun_out/r2w
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -k valley -m gpu -q --timeout 120 --timeout-method thread > $OUT/shard.log 2>&1
tail -3 $OUT/shard.log
MMBA_PROBE=1 timeout -k 10 120 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/probe.json 2> $OUT/probe.err || exit 1
grep "mmba probe" $OUT/probe.err
MMBA_PROBE=1 MMBA_BCR_DF=0 timeout -k 10 120 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/probe0.json 2> $OUT/probe0.err || exit 1
grep "mmba probe" $OUT/probe0.err
echo done
