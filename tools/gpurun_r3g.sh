# full GPU suite (JB in bundle order, nloc once, two-wave potf64, hand dgemm), C3 A/B, C4 bench
set -o pipefail
OUT=gpurun_out/r3g
mkdir -p $OUT
MAXFAIL=30 bash tools/gpurun_tests.sh $OUT tests > /dev/null 2>&1 || echo "TESTS FAILED"
grep -E "FAILED|passed|failed" $OUT/tests.log | tail -30
for h in 1 0; do
  MMBA_DENSE_HAND=$h timeout -k 10 300 python -u bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_h$h.json 2> $OUT/c3_h$h.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/c3_h$h.json').read()); c=d['reduced_cholesky']; print('hand=$h C3 it/s', d['lm_iterations_per_s'], 'ms/solve', d['ms_per_step'], 'chol ms', c['avg_ms'], 'TF', c.get('achieved_tflops'), 'frac', c.get('frac'), 'rms', d['final_rms_px'], 'iters', d['lm_iterations_per_solve'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c3 -- python3 bench.py --config 2 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/c3_prof.json 2> $OUT/c3_prof.err || exit 1
python3 tools/kstats.py $OUT/prof/c3_kernel_stats.csv 8; rm -f $OUT/prof/c3_kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c4_prof.json 2> $OUT/c4_prof.err || exit 1
python3 tools/kstats.py $OUT/prof/c4_kernel_stats.csv 14; rm -f $OUT/prof/c4_kernel_trace.csv
python3 -c "
import json; d=json.loads(open('$OUT/c4_prof.json').read()); print('C4 it/s', d['lm_iterations_per_s'], 'K2 ms', d['roofline']['avg_ms'], 'frac', d['roofline']['frac'], 'chol ms', d['reduced_cholesky']['avg_ms'])"
echo done
