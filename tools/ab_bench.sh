# A/B wall-clock: one bench line per variant (no profiler), interleaved reps.
# A variant is a string of extra bench.py arguments, normally path pins:
# usage: CFGS="1 3" REPS=2 STEPS=20 bash tools/ab_bench.sh <outdir> "" "--path pcr=0" ...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
CFGS=${CFGS:-3}; REPS=${REPS:-1}; STEPS=${STEPS:-10}
for r in $(seq 1 $REPS); do
  for c in $CFGS; do
    i=0
    for e in "$@"; do
      timeout -k 10 200 python -u bench.py $e --config $c --steps $STEPS --warmup 2 --no-cpu-baseline --no-traffic > $OUT/c${c}_v${i}_r$r.json 2> $OUT/c${c}_v${i}_r$r.err || exit 1
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c%s %-28s r%s  %8.1f it/s  %7.3f ms/step  pcie %8.1f it/s' % (sys.argv[2], sys.argv[3], sys.argv[4], d['lm_iterations_per_s'], d['ms_per_step'], d.get('pcie_inclusive', {}).get('lm_iterations_per_s', 0)))" $OUT/c${c}_v${i}_r$r.json $c "$e" $r | tee -a $OUT/summary.txt
      i=$((i+1))
    done
  done
done
echo done
