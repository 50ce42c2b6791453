# rebuilt tree (header fix): full GPU suite + smoke + default bench
set -o pipefail
OUT=gpurun_out/r4e
mkdir -p $OUT
MAXFAIL=30 bash tools/gpurun_tests.sh $OUT tests > /dev/null 2>&1 || echo "TESTS FAILED"
grep -E "FAILED|passed|failed" $OUT/tests.log | tail -10
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
cat $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/default.json 2> $OUT/default.err || exit 1
python3 -c "
import json; d=json.loads(open('$OUT/default.json').read()); r=d['roofline']; print('default C4 it/s %.1f value %.4g K2 frac %.4f traffic %.4g chol ms %.4f' % (d['lm_iterations_per_s'], d['value'], r['frac'], r['traffic'] or 0, d['reduced_cholesky']['avg_ms']))"
