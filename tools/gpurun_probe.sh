# Parity tests, then band-kernel phase probes for C4/C2 at block 8 and 16.
set -o pipefail
OUT=gpurun_out/probe
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed" >> $OUT/tests.log; exit 1; }
for nb in 8 16; do
  for c in 3 1; do
    MMBA_BAND_NB=$nb MMBA_PROBE=1 timeout -k 10 200 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_${c}_nb$nb.json 2> $OUT/bench_${c}_nb$nb.err || exit 1
  done
done
echo done
