# C5 with the rolling shutter (rs 0.5): the library build against a two-wave
# k_jacobian_rs build (tools/libmmba_rs2.so, MMBA_RS_WAVES=2)
set -o pipefail
OUT=${1:-gpurun_out/r5_rs}
mkdir -p $OUT
for v in base rs2 base rs2; do
  MMBA_LIB=$PWD/tools/libmmba_$v.so timeout -k 10 300 python -u bench.py --config 4 --rolling-shutter 0.5 --steps 6 --warmup 2 --no-cpu-baseline --no-traffic > $OUT/c5rs_$v.json 2> $OUT/c5rs_$v.err || { tail $OUT/c5rs_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5rs_$v.json')); print('$v', d['ms_per_step'], d['lm_iterations_per_s'])"
done
