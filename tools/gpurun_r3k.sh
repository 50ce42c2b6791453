set -o pipefail
OUT=gpurun_out/r3k
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_sharded.py -k "dgemm or rccl or local_group" -m gpu -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -15 $OUT/tests.log; exit $rc
