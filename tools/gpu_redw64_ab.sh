# C4: k_schur_obs's reduction workgroups with every load issued first
# (tools/libmmba_new.so) against the load-per-iteration loop (base)
set -o pipefail
OUT=${1:-gpurun_out/r5_redw64}
mkdir -p $OUT
for v in base new base new; do
  MMBA_LIB=$PWD/tools/libmmba_$v.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/c4_$v.json 2> $OUT/c4_$v.err || { tail $OUT/c4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4_$v.json')); print('$v', d['ms_per_step'], d['lm_iterations_per_s'])"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "steps or config_parity or bcr or golden or full_size" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; exit $rc
