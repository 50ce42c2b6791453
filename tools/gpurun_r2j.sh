# BCR register pivot chain A/B + band/plan-cache tests
set -o pipefail
OUT=gpurun_out/r2j
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MAXFAIL=10 bash tools/gpurun_tests.sh $OUT tests/test_gpu_band.py tests/test_gpu_plan_cache.py tests/test_gpu_parity.py || exit 1
for rc in 1 0; do
  MMBA_BCR_REGCHOL=$rc timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_reg$rc.json 2> $OUT/c3_reg$rc.err || exit 1
  cut -c1-700 $OUT/c3_reg$rc.json
  MMBA_BCR_REGCHOL=$rc timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$rc -o c4 -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > /dev/null 2> $OUT/prof$rc.err || exit 1
  grep -E "k_bcr" $OUT/prof$rc/c4_kernel_stats.csv | cut -c1-140
done
echo done
