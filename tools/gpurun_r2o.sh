# DNORM from the speculative trial + bundle factor folded into k_schur_obs: suite + C4/C2/C5 + A/B
set -o pipefail
OUT=gpurun_out/r2o
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MAXFAIL=20 bash tools/gpurun_tests.sh $OUT tests || exit 1
for c in 3 1 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  grep -o '"workload": "[a-z0-9_]*"\|"ms_per_step": [0-9.]*\|"lm_iterations_per_s": [0-9.]*\|"lm_iterations_per_solve": [0-9]*' $OUT/c$c.json | tr '\n' ' '; echo
done
MMBA_BUNDLE_FACTOR_FUSED=0 timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_split.json 2> $OUT/c3_split.err || exit 1
grep -o '"ms_per_step": [0-9.]*\|"lm_iterations_per_s": [0-9.]*\|"lm_iterations_per_solve": [0-9]*' $OUT/c3_split.json | tr '\n' ' '; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > /dev/null 2> $OUT/prof.err || exit 1
head -24 $OUT/prof/c4_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
