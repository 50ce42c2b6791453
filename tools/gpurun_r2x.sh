# BCR chain microbenchmark + finer item phase probe
set -o pipefail
OUT=gpurun_out/r2x
mkdir -p $OUT
timeout -k 10 60 ./tools/ubench/bcr_chain > $OUT/chain.txt 2>&1 || exit 1
cat $OUT/chain.txt
MMBA_PROBE=1 timeout -k 10 120 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/probe.json 2> $OUT/probe.err || exit 1
grep "mmba probe" $OUT/probe.err
echo done
