# C5: the camera-frame normal equations with one wave per camera-frame
# (tools/libmmba_base.so) against four (tools/libmmba_wide.so)
set -o pipefail
OUT=${1:-gpurun_out/r5_ne}
mkdir -p $OUT
for v in base wide base wide; do
  MMBA_LIB=$PWD/tools/libmmba_$v.so timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail $OUT/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5_$v.json')); print('$v', d['ms_per_step'], d['lm_iterations_per_s'])"
done
