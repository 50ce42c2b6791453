# One GPU cycle: parity tests, bench lines for C4/C2/C5, rocprof kernel stats of C4.
set -o pipefail
OUT=gpurun_out/cycle
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed" >> $OUT/tests.log; exit 1; }
for c in 3 1 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err || exit 1
echo "all done"
