# XCD-contiguous split K2 (C2 path): parity subset + C2/C5 lines + C2 kernel stats
set -o pipefail
OUT=gpurun_out/r4b
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_edge.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for c in 1 4 1 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-traffic > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/c$c.json').read()); print('config $c it/s %.1f K2 ms %.4f' % (d['lm_iterations_per_s'], d['roofline']['avg_ms']))"
done
