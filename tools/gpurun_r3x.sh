# XCD-contiguous records / residual blocks: parity subset + C4 kernel stats
set -o pipefail
OUT=gpurun_out/r3z
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_bcr_variants.py tests/test_gpu_plan_cache.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c4.json 2> $OUT/c4.err || exit 1
python3 tools/kstats.py $OUT/prof/c4_kernel_stats.csv 10; rm -f $OUT/prof/c4_kernel_trace.csv
for i in 1 2; do
timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c4_$i.json 2> $OUT/c4_$i.err || exit 1
python3 -c "
import json; d=json.loads(open('$OUT/c4_$i.json').read()); print('C4 it/s %.1f K2 ms %.4f' % (d['lm_iterations_per_s'], d['roofline']['avg_ms']))"
done
