# C3: kernel statistics of one solve (rocprofv3 --kernel-trace --stats)
set -o pipefail
OUT=${1:-gpurun_out/r5_c3}
mkdir -p $OUT
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c3 --output-format csv -- python3 bench.py --config 2 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
python3 - $OUT > $OUT/c3_summary.txt <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1] + '/prof/c3_kernel_stats.csv')))
tot = sum(float(x['TotalDurationNs']) for x in r)
for x in r[:25]:
    print(x['Name'][:70].ljust(70), x['Calls'], round(float(x['AverageNs']) / 1e3, 2), round(float(x['TotalDurationNs']) / 1e6, 2), round(float(x['TotalDurationNs']) / tot * 100, 1))
PY
rm -f $OUT/prof/*kernel_trace* $OUT/prof/*.db
cat $OUT/c3_summary.txt
