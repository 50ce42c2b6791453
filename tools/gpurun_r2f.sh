# direct block-diagonal solve + merged synchronisations: GPU suite, then C2/C5/C4 bench lines
set -o pipefail
OUT=gpurun_out/r2f
mkdir -p $OUT
MAXFAIL=30 bash tools/gpurun_tests.sh $OUT tests || exit 1
for c in 1 4 3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  cat $OUT/c$c.json
done
echo done
