# fused K2 wave-count check on C4 (+ C2 split path) with PMC traffic
set -o pipefail
OUT=gpurun_out/r2h
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || exit 1
cat $OUT/c3.json
timeout -k 10 300 python -u bench.py --config 1 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c1.json 2> $OUT/c1.err || exit 1
cat $OUT/c1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c3_prof.json 2> $OUT/c3_prof.err || exit 1
grep -E "k_jac_ne|k_ne_bnd" $OUT/prof/c4_kernel_stats.csv
echo done
