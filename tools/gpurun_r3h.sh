# dense trailing-update block width A/B (256 vs 512) for the hand kernel and rocBLAS
set -o pipefail
OUT=gpurun_out/r3h
mkdir -p $OUT
for nb in 512 256; do for h in 1 0; do
  MMBA_DENSE_NB=$nb MMBA_DENSE_HAND=$h timeout -k 10 300 python -u bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_nb${nb}_h$h.json 2> $OUT/c3_nb${nb}_h$h.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/c3_nb${nb}_h$h.json').read()); c=d['reduced_cholesky']; print('nb=$nb hand=$h C3 it/s %.3f chol ms %.1f TF %.2f frac %.3f rms %.6f iters %d' % (d['lm_iterations_per_s'], c['avg_ms'], c.get('achieved_tflops'), c.get('frac'), d['final_rms_px'], d['lm_iterations_per_solve']))"
done; done
echo done
