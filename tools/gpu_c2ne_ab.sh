# C2: k_ne_cf_u with sixteen waves per camera-frame (measured slower and not kept:
# profiles/r5_c2ne/) against four; then the GPU suite
set -o pipefail
OUT=${1:-gpurun_out/r5_c2ne}
mkdir -p $OUT
for v in base new base new; do
  MMBA_LIB=$PWD/tools/libmmba_$v.so timeout -k 10 300 python -u bench.py --config 1 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/c2_$v.json 2> $OUT/c2_$v.err || { tail $OUT/c2_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c2_$v.json')); print('$v', d['ms_per_step'], d['lm_iterations_per_s'], d['device_resident']['lm_iterations_per_s'], d['roofline']['avg_ms'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; exit $rc
