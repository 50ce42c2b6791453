# C2 all-frames kernel timeline
set -o pipefail
OUT=gpurun_out/r2e
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof -o c2 -- python3 bench.py --config 1 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c2.json 2> $OUT/c2.err || exit 1
cat $OUT/c2.json
