set -o pipefail
mkdir -p gpurun_out/r1_s7e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1_s7e/gpu_tests.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r1_s7e/bench_c4.json 2> gpurun_out/r1_s7e/bench_c4.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r1_s7e/prof -o c4 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1_s7e/prof_bench.json 2> gpurun_out/r1_s7e/prof_bench.err
echo "exit=$?"
