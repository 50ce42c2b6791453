# RS tests + golden (RS fixture) + C5-RS bench + profile of C5-RS
set -o pipefail
OUT=${1:-gpurun_out/rs}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rs.py tests/test_gpu_golden.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -15 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
ROOT=$(pwd); cd /tmp && cd $ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5rs -o c5rs --output-format csv -- python3 bench.py --config 4 --rolling-shutter 0.5 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c5rs.json 2> $OUT/c5rs.err || { tail $OUT/c5rs.err; exit 1; }
rm -f $OUT/c5rs/c5rs_kernel_trace.csv
python3 tools/kstats.py $OUT/c5rs/c5rs_kernel_stats.csv > $OUT/c5rs_summary.txt
cat $OUT/c5rs_summary.txt; cat $OUT/c5rs.json
