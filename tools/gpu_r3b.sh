# whole GPU suite (incl. RS, shim, full-size), shim executable, C5-RS / C5 / C4 bench lines
set -o pipefail
OUT=gpurun_out/r3c
mkdir -p $OUT
make -s -C tests/shim || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -30 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tests/shim/shim_core_test > $OUT/shim.log 2>&1; rc=$?; cat $OUT/shim.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config 4 --rolling-shutter 0.5 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench_c5rs.json 2> $OUT/bench_c5rs.err || { tail $OUT/bench_c5rs.err; exit 1; }
cat $OUT/bench_c5rs.json
timeout -k 10 300 python -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 1
cat $OUT/bench_c5.json
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 1
cat $OUT/bench_c4.json
