# dataflow BCR factor: variant bitwise tests + band tests, then the full GPU
# suite, C4 A/B (dataflow vs per-level) with kernel stats, the default bench
set -o pipefail
OUT=gpurun_out/r2r
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bcr_variants.py tests/test_gpu_band.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/bcr_tests.log 2>&1
rc=$?; tail -15 $OUT/bcr_tests.log; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for df in 1 0; do
  MMBA_BCR_DF=$df timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$df -o c4 -- python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c4_df$df.json 2> $OUT/c4_df$df.err || exit 1
  cat $OUT/c4_df$df.json
  grep -E "bcr" $OUT/p$df/c4_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
MAXFAIL=30 bash tools/gpurun_tests.sh $OUT tests || echo "TESTS FAILED"
grep -E "FAILED|passed|failed" $OUT/tests.log | tail -40
timeout -k 10 600 python -u bench.py > $OUT/default.json 2> $OUT/default.err || exit 1
cat $OUT/default.json
for c in 1 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  cat $OUT/c$c.json
done
echo done
