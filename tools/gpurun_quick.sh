# Quick GPU cycle: parity tests, C4/C2/C5 bench lines (no CPU baseline, no PMC),
# rocprofv3 kernel stats of C4, optional MMBA_PROBE run.
# usage: bash tools/gpurun_quick.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed" >> $OUT/tests.log; exit 1; }
for c in 3 1 4; do
  timeout -k 10 200 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/prof_bench.json 2> $OUT/prof_bench.err || exit 1
if [ -n "$PROBE" ]; then
  MMBA_PROBE=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/probe.json 2> $OUT/probe.err || exit 1
fi
echo "all done"
