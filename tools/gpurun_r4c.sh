# final round-2 state: full GPU suite, smoke, default bench line (PMC + CPU baseline),
# rocprof stats of the default command, BCR probe, C2/C5/C1 lines
set -o pipefail
OUT=gpurun_out/r4c
mkdir -p $OUT
MAXFAIL=30 bash tools/gpurun_tests.sh $OUT tests > /dev/null 2>&1 || echo "TESTS FAILED"
grep -E "FAILED|passed|failed" $OUT/tests.log | tail -30
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
cat $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/default.json 2> $OUT/default.err || exit 1
python3 -c "
import json; d=json.loads(open('$OUT/default.json').read()); r=d['roofline']; c=d['reduced_cholesky']; print('default C4 it/s %.1f value %.4g ms/step %.2f K2 ms %.4f frac %.4f traffic %.4g chol ms %.4f cpu %s' % (d['lm_iterations_per_s'], d['value'], d['ms_per_step'], r['avg_ms'], r['frac'], r['traffic'] or 0, c['avg_ms'], d['cpu_baseline'] and d['cpu_baseline']['value']))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o default -- python3 bench.py --no-cpu-baseline --no-traffic > $OUT/default_prof.json 2> $OUT/default_prof.err || exit 1
python3 tools/kstats.py $OUT/prof/default_kernel_stats.csv 20; rm -f $OUT/prof/default_kernel_trace.csv
MMBA_PROBE=1 timeout -k 10 120 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/probe.json 2> $OUT/probe.err || exit 1
grep "mmba probe" $OUT/probe.err
for c in 0 1 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-traffic > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/c$c.json').read()); print('config $c', d['config']['workload'], 'it/s %.1f ms/solve %.3f resid/s %.3g rms %.4f' % (d['lm_iterations_per_s'], d['ms_per_step'], d['value'], d['final_rms_px']))"
done
echo done
