# A/B wall-clock: C4 bench line per env setting (no profiler).
# usage: bash tools/ab_bench.sh <outdir> "ENV=a" "ENV=b" ...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
i=0
for e in "$@"; do
  env $e timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/b$i.json 2> $OUT/b$i.err || exit 1
  echo "$e" > $OUT/env$i.txt
  i=$((i+1))
done
echo done
