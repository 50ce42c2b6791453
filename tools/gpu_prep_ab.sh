# C5: the trial point's parameter pass + k_records (--path trial_records=0)
# against k_trial_prep_rec (default), then the GPU suite
set -o pipefail
OUT=${1:-gpurun_out/r5_prep}
mkdir -p $OUT
for v in off on off on; do
  P=""; [ $v = off ] && P="--path trial_records=0"
  timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic $P > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail $OUT/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5_$v.json')); print('$v', d['ms_per_step'], d['lm_iterations_per_s'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; exit $rc
