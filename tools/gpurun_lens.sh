# GPU cycle for the lens models: all GPU tests, C5 bench lines (classic, radial).
set -o pipefail
OUT=${1:-gpurun_out/lens}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed" >> $OUT/tests.log; tail -30 $OUT/tests.log; exit 1; }
timeout -k 10 200 python -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench_4.json 2> $OUT/bench_4.err || exit 1
timeout -k 10 200 python -u bench.py --config 4 --lens-model radial --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench_4r.json 2> $OUT/bench_4r.err || exit 1
timeout -k 10 200 python -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench_3.json 2> $OUT/bench_3.err || exit 1
echo "all done"
