# Profile configs other than C4: kernel trace of C2 and C5, and one full-size C3 solve.
set -o pipefail
OUT=${1:-gpurun_out/cfg}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in 1 4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof$c -o c$c --output-format csv -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/prof$c.json 2> $OUT/prof$c.err || exit 1
done
timeout -k 10 400 python -u bench.py --config 2 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/bench_2.json 2> $OUT/bench_2.err || exit 1
echo done
