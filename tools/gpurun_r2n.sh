# MFMA BCR updates + sharded epilogue/collective folding: full GPU suite, C4 A/B, probe, chain ubench
set -o pipefail
OUT=gpurun_out/r2n
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 5 60 ./tools/ubench/chain > $OUT/chain.txt 2>&1 || exit 1
cat $OUT/chain.txt
MAXFAIL=20 bash tools/gpurun_tests.sh $OUT tests || exit 1
for mf in 1 0; do
  MMBA_BCR_MFMA=$mf timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_mf$mf.json 2> $OUT/c3_mf$mf.err || exit 1
  grep -o '"ms_per_step": [0-9.]*\|"lm_iterations_per_s": [0-9.]*\|"lm_iterations_per_solve": [0-9]*' $OUT/c3_mf$mf.json
  grep -o '"reduced_cholesky": {"avg_ms": [0-9.]*' $OUT/c3_mf$mf.json
  MMBA_PROBE=1 MMBA_BCR_MFMA=$mf timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > /dev/null 2> $OUT/probe$mf.err || exit 1
  grep -a "mmba probe" $OUT/probe$mf.err
done
