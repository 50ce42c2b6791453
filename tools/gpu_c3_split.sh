# (round 5 record: the dense_split path key was removed after this measurement --
# profiles/r5_c3split/; the script no longer runs against the current library)
# C3: the dense factorisation with its panel chain on a CU partition
# (--path dense_split=V) against the single-stream form
set -o pipefail
OUT=${1:-gpurun_out/r5_c3split}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "dense_split or dense_and_tiled" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in 0 32 4128 16 64; do
  timeout -k 10 300 python -u bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic --path dense_split=$v > $OUT/c3_$v.json 2> $OUT/c3_$v.err || { tail $OUT/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c3_$v.json')); print('$v', d['ms_per_step'], d['lm_iterations_per_s'], d['reduced_cholesky']['avg_ms'], d['final_rms_px'], d['reason_number'])"
done
