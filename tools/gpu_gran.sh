set -o pipefail
OUT=${1:-gpurun_out/r5_gran}
mkdir -p $OUT
(cd tools/ubench && timeout -k 10 60 ./pcr_probe 2994 > ../../$OUT/probe.txt 2>&1) || { cat $OUT/probe.txt; exit 1; }
cat $OUT/probe.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bcr or band or pcr or steps or sharded or group" > $OUT/tests.log 2>&1; rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['lm_iterations_per_s'], d['reduced_cholesky']['avg_ms'])"
