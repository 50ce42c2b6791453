# Dense/tiled parity tests, then the kernel stats of one full-size C3 solve.
set -o pipefail
OUT=${1:-gpurun_out/c3p}
mkdir -p $OUT
[ -n "$SKIP_TESTS" ] || { timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "dense or config" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }; }
tail -2 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c3 --output-format csv -- python3 bench.py --config 2 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/prof.json 2> $OUT/prof.err || exit 1
rm -f $OUT/prof/*kernel_trace.csv
echo done
