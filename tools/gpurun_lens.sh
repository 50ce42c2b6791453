# GPU cycle for the lens models: all GPU tests, C5 bench lines per lens model.
set -o pipefail
OUT=${1:-gpurun_out/lens}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed" >> $OUT/tests.log; tail -30 $OUT/tests.log; exit 1; }
for lm in classic radial anamorphic anamorphic_rescaled; do
  timeout -k 10 200 python -u bench.py --config 4 --lens-model $lm --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench_4_$lm.json 2> $OUT/bench_4_$lm.err || exit 1
done
echo "all done"
