set -o pipefail
OUT=gpurun_out/r5_jac
mkdir -p $OUT
for v in base jac_occ1 jac_occ2 base jac_occ2; do
  MMBA_LIB=$PWD/tools/libmmba_$v.so timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { tail $OUT/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c5_$v.json')); print('$v', d['ms_per_step'], d['lm_iterations_per_s'])"
done
