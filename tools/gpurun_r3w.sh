# SQ counters (one pass) for the C4 kernels: where the BCR and K2 waves spend their cycles
set -o pipefail
OUT=gpurun_out/r3w
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT/pmc -o sq -- python3 bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/sq.json 2> $OUT/sq.err || exit 1
ls $OUT/pmc
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/r3w/pmc/*counter_collection.csv')[0]
rows = list(csv.DictReader(open(f)))
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r['Kernel_Name'].split('(')[0]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Counter_Name'])] += 1
out = []
for k, d in acc.items():
    disp = max(n[(k, c)] for c in d)
    w = d.get('SQ_WAVE_CYCLES', 0)
    if w <= 0: continue
    out.append((w, k, d, disp))
out.sort(reverse=True)
with open('gpurun_out/r3w/sq_summary.txt', 'w') as fo:
    for w, k, d, disp in out[:12]:
        line = '%-40s disp=%4d wave_cyc/disp=%10.0f  active %4.1f%%  wait_any %4.1f%%  wait_inst %4.1f%% (lds %4.1f%%)  VALU/disp %8.0f LDS/disp %7.0f SALU/disp %7.0f' % (
            k[-40:], disp, w / disp, 100 * d['SQ_ACTIVE_INST_ANY'] / w, 100 * d['SQ_WAIT_ANY'] / w,
            100 * d['SQ_WAIT_INST_ANY'] / w, 100 * d['SQ_WAIT_INST_LDS'] / w, d['SQ_INSTS_VALU'] / disp,
            d['SQ_INSTS_LDS'] / disp, d['SQ_INSTS_SALU'] / disp)
        print(line); fo.write(line + '\n')
PY
rm -f $OUT/pmc/*counter_collection.csv
