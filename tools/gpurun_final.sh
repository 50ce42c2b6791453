# Round-end style cycle: all GPU tests, smoke(), default bench (CPU baseline +
# PMC traffic), C2/C3/C5 bench lines, rocprofv3 stats + one-iteration trace of C4.
set -o pipefail
OUT=${1:-gpurun_out/final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed" >> $OUT/tests.log; tail -30 $OUT/tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $OUT/bench_3.json 2> $OUT/bench_3.err || exit 1
for c in 1 4; do
  timeout -k 10 200 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
done
timeout -k 10 400 python -u bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench_2.json 2> $OUT/bench_2.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/prof_bench.json 2> $OUT/prof_bench.err || exit 1
python3 tools/iter_trace.py $OUT/prof/c4_kernel_trace.csv > $OUT/c4_iteration_trace.txt && rm -f $OUT/prof/c4_kernel_trace.csv
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_schur_dest_u|k_residual|k_jacobian_u" -d $OUT/pmc_fetch -o c4 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_schur_dest_u|k_residual|k_jacobian_u" -d $OUT/pmc_write -o c4 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit 1
echo "all done"
