# C4 / C2 bench lines (two rounds) on the current tree
set -o pipefail
OUT=${1:-gpurun_out/fab}
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-traffic > $OUT/c4_$r.json 2> $OUT/c4_$r.err || exit 1
  timeout -k 10 300 python3 bench.py --config 1 --steps 12 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/c1_$r.json 2> $OUT/c1_$r.err || exit 1
done
python3 - $OUT <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    print("%-8s %8.0f LM it/s  device-resident %8.0f  ms/solve %.3f" % (f.split("/")[-1][:-5], d["lm_iterations_per_s"], d["device_resident"]["lm_iterations_per_s"], d["ms_per_step"]))
PY
