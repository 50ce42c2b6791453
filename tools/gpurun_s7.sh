set -o pipefail
mkdir -p gpurun_out/r1_s7
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1_s7/gpu_tests.txt 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r1_s7/smoke.txt 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r1_s7/bench_default.json 2> gpurun_out/r1_s7/bench_default.err
echo "exit=$?"
