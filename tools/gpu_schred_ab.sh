# The Jacobian epilogue's row reductions inside the next damped solve's first
# launch (k_schur_init on C5, k_schur_obs on C4; tools/libmmba_new.so) against
# their own k_reduce_multi launch (tools/libmmba_base.so); then the GPU suite
set -o pipefail
OUT=${1:-gpurun_out/r5_schred}
mkdir -p $OUT
for cfg in 4 3; do
for v in base new base new; do
  MMBA_LIB=$PWD/tools/libmmba_$v.so timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/c${cfg}_$v.json 2> $OUT/c${cfg}_$v.err || { tail $OUT/c${cfg}_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c${cfg}_$v.json')); print('cfg $cfg $v', d['ms_per_step'], d['lm_iterations_per_s'])"
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; exit $rc
