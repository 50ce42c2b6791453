set -o pipefail
OUT=gpurun_out/r3t
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c2 -- python3 bench.py --config 1 --steps 20 --warmup 2 --no-cpu-baseline --no-traffic > $OUT/c2.json 2> $OUT/c2.err || exit 1
python3 tools/kstats.py $OUT/prof/c2_kernel_stats.csv 25
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r3t/prof/c2_kernel_trace.csv')))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
# gaps between consecutive kernels in the last 200 launches
st=[int(r['Start_Timestamp']) for r in rows][-300:]; en=[int(r['End_Timestamp']) for r in rows][-300:]
nm=[r['Kernel_Name'].split('(')[0][-30:] for r in rows][-300:]
gaps=[st[i+1]-en[i] for i in range(len(st)-1)]
import statistics
print('launches', len(rows), 'median gap us %.2f' % (statistics.median(gaps)/1e3), 'mean gap %.2f' % (sum(gaps)/len(gaps)/1e3))
big=sorted(range(len(gaps)), key=lambda i:-gaps[i])[:8]
for i in big: print('gap %.1f us after %s before %s' % (gaps[i]/1e3, nm[i], nm[i+1]))
for i in range(-40,0): print('%-30s dur %.1f gap-before %.1f' % (nm[i], (en[i]-st[i])/1e3, (st[i]-en[i-1])/1e3))
PY
rm -f $OUT/prof/c2_kernel_trace.csv
cat $OUT/c2.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('C2 it/s', d['lm_iterations_per_s'], d['time_split_s'])"
