# re-entry verification: full GPU suite, smoke, default bench, C4 kernel stats
set -o pipefail
OUT=gpurun_out/r2v
mkdir -p $OUT
MAXFAIL=30 bash tools/gpurun_tests.sh $OUT tests || echo "TESTS FAILED"
grep -E "FAILED|passed|failed" $OUT/tests.log | tail -40
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
cat $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/default.json 2> $OUT/default.err || exit 1
cat $OUT/default.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c4_prof.json 2> $OUT/c4_prof.err || exit 1
cat $OUT/c4_prof.json
for c in 1 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  cat $OUT/c$c.json
done
echo done
