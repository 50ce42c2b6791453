# C2 per-frame bench (cached plan, one launch per call) + kernel trace
set -o pipefail
OUT=gpurun_out/r2d
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --config 1 --per-frame 64 --steps 10 --warmup 2 > $OUT/c1_pf.json 2> $OUT/c1_pf.err || exit 1
cat $OUT/c1_pf.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o pf -- python3 bench.py --config 1 --per-frame 64 --steps 10 --warmup 2 > $OUT/c1_pf_prof.json 2> $OUT/c1_pf_prof.err || exit 1
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs head -8
