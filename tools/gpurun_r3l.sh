# BCR chains without per-step pivot checks: item ubench, BCR/band/golden/parity/sharded tests, C4 bench
set -o pipefail
OUT=gpurun_out/r3n
mkdir -p $OUT
true
true
timeout -k 10 500 python -u -m pytest tests/test_gpu_bcr_variants.py tests/test_gpu_band.py tests/test_gpu_golden.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c4_$i.json 2> $OUT/c4_$i.err || exit 1
python3 -c "
import json; d=json.loads(open('$OUT/c4_$i.json').read()); print('C4 it/s %.1f chol ms %.4f K2 ms %.4f' % (d['lm_iterations_per_s'], d['reduced_cholesky']['avg_ms'], d['roofline']['avg_ms']))"
done
echo done
