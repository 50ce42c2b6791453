# BCR level phase probe (MMBA_PROBE=1), LDS vs register pivot chain
set -o pipefail
OUT=gpurun_out/r2k
mkdir -p $OUT
for rc in 0 1; do
  MMBA_PROBE=1 MMBA_BCR_REGCHOL=$rc timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/c3_reg$rc.json 2> $OUT/c3_reg$rc.err || exit 1
  grep -a "mmba probe" $OUT/c3_reg$rc.err
done
