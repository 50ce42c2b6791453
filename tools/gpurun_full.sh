# Full GPU cycle: parity tests, C4 bench (with CPU baseline), C2/C5 bench lines,
# rocprofv3 kernel stats of the C4 bench, and two PMC passes (FETCH_SIZE,
# WRITE_SIZE) over the K2 kernels for the roofline `traffic` field.
# usage: bash tools/gpurun_full.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/full}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed" >> $OUT/tests.log; exit 1; }
timeout -k 10 300 python -u bench.py $BENCH3_ARGS > $OUT/bench_3.json 2> $OUT/bench_3.err || exit 1
for c in 1 4; do
  timeout -k 10 200 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err || exit 1
[ -n "$NO_PMC" ] && { echo "all done (no pmc)"; exit 0; }
REGEX=${MMBA_PMC_REGEX:-k_jacobian|k_ne_|k_residual|k_schur_dest|k_band_factor}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$REGEX" -d $OUT/pmc_fetch -o c4 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$REGEX" -d $OUT/pmc_write -o c4 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit 1
echo "all done"
