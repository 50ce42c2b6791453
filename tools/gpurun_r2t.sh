set -o pipefail
OUT=gpurun_out/r2t
mkdir -p $OUT
timeout -k 10 120 python -u tools/debug_bcr_df.py 6 > $OUT/df.log 2>&1 || exit 1
MMBA_BCR_DF=0 timeout -k 10 120 python -u tools/debug_bcr_df.py 6 > $OUT/lv.log 2>&1 || exit 1
cat $OUT/df.log $OUT/lv.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_bcr_variants.py tests/test_gpu_plan_cache.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/bcr_tests.log 2>&1
tail -5 $OUT/bcr_tests.log
