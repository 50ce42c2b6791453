# fused K2: GPU suite, C2/C5 lines, C4 with PMC traffic, K2 A/B (MMBA_K2_FUSED=0)
set -o pipefail
OUT=gpurun_out/r2g
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MAXFAIL=30 bash tools/gpurun_tests.sh $OUT tests || exit 1
for c in 1 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  cat $OUT/c$c.json
done
timeout -k 10 600 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || exit 1
cat $OUT/c3.json
MMBA_K2_FUSED=0 timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_split.json 2> $OUT/c3_split.err || exit 1
cat $OUT/c3_split.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_prof.json 2> $OUT/c3_prof.err || exit 1
head -20 $OUT/prof/c4_kernel_stats.csv
echo done
