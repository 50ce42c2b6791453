set -o pipefail
O=gpurun_out/r3g; mkdir -p $O
MMBA_LM_COOP=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "coop or full_size or perframe or golden" > $O/tests_coop.log 2>&1 || { tail -40 $O/tests_coop.log; exit 1; }
tail -2 $O/tests_coop.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_bench_env.sh $O c4_prejac 3 && bash tools/gpu_bench_env.sh $O c4_noprejac 3 MMBA_PRE_JAC=0 && bash tools/gpu_bench_env.sh $O c4_prejac_seq 3 MMBA_HOST_MIRROR=1 MMBA_SEQ_POLL=1 && bash tools/gpu_bench_env.sh $O c2_coop 1 MMBA_LM_COOP=1 && bash tools/gpu_bench_env.sh $O c2_host 1
