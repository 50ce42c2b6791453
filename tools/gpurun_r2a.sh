# C2 overhead trace + default bench (new measured cpu_baseline)
set -o pipefail
OUT=gpurun_out/r2a
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/c2prof -o c2 -- python3 bench.py --config 1 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c2_bench.json 2> $OUT/c2_bench.err || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
echo done
