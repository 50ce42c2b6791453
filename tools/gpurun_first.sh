set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -q -rf > gpurun_out/t2.log 2>&1
echo "exit=$?" >> gpurun_out/t2.log
