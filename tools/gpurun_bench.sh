set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
echo "exit=$?" >> gpurun_out/bench_c4.err
timeout -k 10 300 python -u bench.py --config 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
timeout -k 10 300 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
echo done
