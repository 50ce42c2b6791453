# round-2 validation after the 4-wave K2: GPU suite (incl. the C4-structure
# x tests), the default bench line (C4 + cpu_baseline + PMC traffic), kernel
# stats, C2 / C5 / C2 per-frame lines
set -o pipefail
OUT=gpurun_out/r2q
mkdir -p $OUT
MAXFAIL=30 bash tools/gpurun_tests.sh $OUT tests || echo "TESTS FAILED rc=$?"
grep -E "FAILED|passed|failed" $OUT/tests.log | tail -40
timeout -k 10 600 python -u bench.py > $OUT/default.json 2> $OUT/default.err || exit 1
cat $OUT/default.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c4_prof.json 2> $OUT/c4_prof.err || exit 1
for c in 1 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  cat $OUT/c$c.json
done
timeout -k 10 300 python -u bench.py --config 1 --per-frame 64 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c1_pf.json 2> $OUT/c1_pf.err || exit 1
cat $OUT/c1_pf.json
echo done
