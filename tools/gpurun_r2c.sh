# batched per-frame LM: per-frame parity tests + the C2 per-frame bench line
set -o pipefail
OUT=gpurun_out/r2c
mkdir -p $OUT
MAXFAIL=20 bash tools/gpurun_tests.sh $OUT tests/test_gpu_perframe.py
rc=$?
timeout -k 10 300 python -u bench.py --config 1 --per-frame 64 --steps 3 --warmup 1 > $OUT/c1_pf.json 2> $OUT/c1_pf.err || exit 1
cat $OUT/c1_pf.json
exit $rc
