# blocked BCR pivot chain: band/parity tests, C4 A/B (MMBA_BCR_CHOL=0/2), probe
set -o pipefail
OUT=gpurun_out/r2l
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MAXFAIL=10 bash tools/gpurun_tests.sh $OUT tests/test_gpu_band.py tests/test_gpu_plan_cache.py tests/test_gpu_parity.py tests/test_gpu_sharded.py || exit 1
for ch in 2 0; do
  MMBA_BCR_CHOL=$ch timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_ch$ch.json 2> $OUT/c3_ch$ch.err || exit 1
  cut -c1-600 $OUT/c3_ch$ch.json | grep -o '"ms_per_step": [0-9.]*\|"lm_iterations_per_s": [0-9.]*\|"lm_iterations_per_solve": [0-9]*\|"avg_ms": [0-9.]*'
  grep -o '"reduced_cholesky": {[^}]*}' $OUT/c3_ch$ch.json
  MMBA_PROBE=1 MMBA_BCR_CHOL=$ch timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > /dev/null 2> $OUT/probe$ch.err || exit 1
  grep -a "mmba probe" $OUT/probe$ch.err
done
