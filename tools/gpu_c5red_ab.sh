# C5: the generic Jacobian epilogue's row reductions inside the k_schur_init
# launch (tools/libmmba_new.so) against their own launch (base); GPU suite
set -o pipefail
OUT=${1:-gpurun_out/r5_c5red}
mkdir -p $OUT
for v in base new base new; do
  MMBA_LIB=$PWD/tools/libmmba_$v.so timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail $OUT/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5_$v.json')); print('$v', d['ms_per_step'], d['lm_iterations_per_s'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; exit $rc
