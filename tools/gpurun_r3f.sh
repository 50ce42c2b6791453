# hand-written fp64 MFMA GEMM/SYRK for the dense reduced solve: parity, C3 A/B, kernel stats
set -o pipefail
OUT=gpurun_out/r3f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "dense or c3" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for h in 1 0; do
  MMBA_DENSE_HAND=$h timeout -k 10 300 python -u bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_h$h.json 2> $OUT/c3_h$h.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/c3_h$h.json').read()); c=d['reduced_cholesky']; print('hand=$h C3 it/s', d['lm_iterations_per_s'], 'ms/solve', d['ms_per_step'], 'chol ms', c['avg_ms'], 'TF', c.get('achieved_tflops'), 'frac', c.get('frac'), 'rms', d['final_rms_px'], 'iters', d['lm_iterations_per_solve'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c3 -- python3 bench.py --config 2 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/c3_prof.json 2> $OUT/c3_prof.err || exit 1
python3 tools/kstats.py $OUT/prof/c3_kernel_stats.csv 8; rm -f $OUT/prof/c3_kernel_trace.csv
echo done
