# MFMA busy counters for the dense reduced solve (C3): k_dgemm_nt MFMA utilisation
set -o pipefail
OUT=gpurun_out/r4d
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc -o c3 -- python3 bench.py --config 2 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/c3.json 2> $OUT/c3.err || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/r4d/pmc/*counter_collection.csv')[0]
rows = list(csv.DictReader(open(f)))
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r['Kernel_Name'].split('(')[0]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Counter_Name'])] += 1
lines = []
for k, d in sorted(acc.items(), key=lambda kv: -kv[1].get('GRBM_GUI_ACTIVE', 0))[:6]:
    g = d.get('GRBM_GUI_ACTIVE', 0)
    mb = d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0)
    util = mb / (g * 1024) if g else 0
    lines.append('%-36s dispatches=%6d GRBM_GUI_ACTIVE=%.4g MFMA_BUSY=%.4g  MFMA busy / (active cycles x 1024 SIMDs) = %.3f' % (
        k[-36:], n[(k, 'GRBM_GUI_ACTIVE')], g, mb, util))
open('gpurun_out/r4d/mfma_summary.txt', 'w').write('\n'.join(lines) + '\n')
print('\n'.join(lines))
PY
rm -f $OUT/pmc/*counter_collection.csv
