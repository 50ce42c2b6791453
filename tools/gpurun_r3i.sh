# round-2 final measurements: smoke, default bench line (PMC traffic + CPU baseline),
# rocprof stats of the same command, C1/C2/C5 lines, per-frame line
set -o pipefail
OUT=gpurun_out/r3i
mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
cat $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/default.json 2> $OUT/default.err || exit 1
cat $OUT/default.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o default -- python3 bench.py --no-cpu-baseline --no-traffic > $OUT/default_prof.json 2> $OUT/default_prof.err || exit 1
python3 tools/kstats.py $OUT/prof/default_kernel_stats.csv 20; rm -f $OUT/prof/default_kernel_trace.csv
for c in 0 1 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-traffic > $OUT/c$c.json 2> $OUT/c$c.err || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/c$c.json').read()); print('config $c', d['config']['workload'], 'it/s %.1f ms/solve %.3f resid/s %.3g rms %.4f' % (d['lm_iterations_per_s'], d['ms_per_step'], d['value'], d['final_rms_px']))"
done
timeout -k 10 300 python -u bench.py --config 1 --per-frame 1 --steps 10 --warmup 2 > $OUT/c1_perframe.json 2> $OUT/c1_perframe.err || exit 1
cat $OUT/c1_perframe.json
echo done
