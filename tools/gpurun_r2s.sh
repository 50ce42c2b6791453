# dataflow BCR: which variant tests differ (no -x)
set -o pipefail
OUT=gpurun_out/r2s
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bcr_variants.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/bcr_tests.log 2>&1
tail -15 $OUT/bcr_tests.log
