# fused K2 waves per camera-frame: 2 / 4 / 8 on C4 (kernel stats)
set -o pipefail
OUT=gpurun_out/r2p
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for nw in 2 4 8; do
  MMBA_K2_WAVES=$nw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$nw -o c4 -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_nw$nw.json 2> $OUT/c3_nw$nw.err || exit 1
  grep -E "k_jac_ne" $OUT/p$nw/c4_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-40,140-200
done
