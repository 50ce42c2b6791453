set -o pipefail
OUT=gpurun_out/r3s
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_bcr_variants.py tests/test_gpu_band.py tests/test_gpu_golden.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
MMBA_PROBE=1 timeout -k 10 120 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/probe.json 2> $OUT/probe.err || exit 1
grep "mmba probe" $OUT/probe.err | tail -3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c4.json 2> $OUT/c4.err || exit 1
python3 tools/kstats.py $OUT/prof/c4_kernel_stats.csv 5; rm -f $OUT/prof/c4_kernel_trace.csv
python3 -c "
import json; d=json.loads(open('$OUT/c4.json').read()); print('C4 it/s %.1f chol ms %.4f' % (d['lm_iterations_per_s'], d['reduced_cholesky']['avg_ms']))"
