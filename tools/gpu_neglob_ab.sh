# C5: k_ne_cf_u + k_ne_glob as one launch (tools/libmmba_new.so) against two
# (tools/libmmba_base.so), then the lens / C5 GPU tests on the new library
set -o pipefail
OUT=${1:-gpurun_out/r5_neglob}
mkdir -p $OUT
for v in base new base new; do
  MMBA_LIB=$PWD/tools/libmmba_$v.so timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail $OUT/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5_$v.json')); print('$v', d['ms_per_step'], d['lm_iterations_per_s'], d['roofline']['avg_ms'])"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "lens or c5 or config_parity or golden or full_size" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; exit $rc
