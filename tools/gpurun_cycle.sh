set -o pipefail
mkdir -p gpurun_out/cycle
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -q -rf -x > gpurun_out/cycle/tests.log 2>&1 || { echo "tests failed" >> gpurun_out/cycle/tests.log; exit 1; }
for c in 3 1 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cycle/bench_$c.json 2> gpurun_out/cycle/bench_$c.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/cycle/prof -o c4 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cycle/prof_bench.json 2> gpurun_out/cycle/prof_bench.err
echo "all done"
