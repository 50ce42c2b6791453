# Parity tests, then C4/C2/C5 bench lines over band partition counts.
set -o pipefail
OUT=gpurun_out/parts
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed" >> $OUT/tests.log; exit 1; }
for P in 1 4 8 12 16 24; do
  MMBA_BAND_PARTS=$P timeout -k 10 200 python -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_3_P$P.json 2> $OUT/bench_3_P$P.err || exit 1
done
for c in 1 4; do
  timeout -k 10 200 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_${c}.json 2> $OUT/bench_${c}.err || exit 1
done
echo done
