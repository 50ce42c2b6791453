# BCR: registers-direct operands + augmented root -- parity subset, probe, C4 bench + kernel stats
set -o pipefail
OUT=gpurun_out/r2z
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
MMBA_PROBE=1 timeout -k 10 120 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/probe.json 2> $OUT/probe.err || exit 1
grep "mmba probe" $OUT/probe.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c4.json 2> $OUT/c4.err || exit 1
cat $OUT/c4.json
grep -E "bcr" $OUT/prof/c4_kernel_stats.csv | cut -d, -f1-5 | cut -c1-150
echo done
