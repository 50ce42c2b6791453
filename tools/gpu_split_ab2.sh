# C2: k_ne_cf_split (default) against k_ne_cf_u (NE_CF_SPLIT=0), alternating, 3 rounds; then a trace of each
set -o pipefail
OUT=${1:-gpurun_out/split2}
mkdir -p $OUT
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python3 bench.py --config 1 --steps 12 --warmup 3 --no-cpu-baseline --no-traffic --path NE_CF_SPLIT=$v > $OUT/s${v}_$r.json 2> $OUT/s${v}_$r.err || exit 1
  done
done
python3 - $OUT <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    print("%-8s %8.0f LM it/s  device-resident %8.0f  ms/solve %.3f" % (f.split("/")[-1][:-5], d["lm_iterations_per_s"], d["device_resident"]["lm_iterations_per_s"], d["ms_per_step"]))
PY
