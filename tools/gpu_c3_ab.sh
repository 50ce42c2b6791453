# C3: the split Schur pass and the eight-lane backward step against the
# wave-per-destination pass (--path dest_lane=0), then the dense / Schur tests
set -o pipefail
OUT=${1:-gpurun_out/r5_c3ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "dest_lane or dense_and_tiled or config_parity" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in on off; do
  P=""; [ $v = off ] && P="--path dest_lane=0"
  timeout -k 10 300 python -u bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic $P > $OUT/c3_$v.json 2> $OUT/c3_$v.err || { tail $OUT/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c3_$v.json')); print('$v', d['ms_per_step'], d['lm_iterations_per_s'], d['reduced_cholesky']['avg_ms'], d['time_split_s'])"
done
