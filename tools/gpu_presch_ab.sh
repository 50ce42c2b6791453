# C4 A/B: k_schur_obs enqueued with the gated Jacobian (default) or after the decision
set -o pipefail
OUT=${1:-gpurun_out/presch}
mkdir -p $OUT
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-traffic --path PRE_SCHUR=$v > $OUT/c4_p${v}_$r.json 2> $OUT/c4_p${v}_$r.err || exit 1
  done
done
python3 - $OUT <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    print("%-10s %8.0f LM it/s  device-resident %8.0f  ms/solve %.3f" % (f.split("/")[-1][:-5], d["lm_iterations_per_s"], d["device_resident"]["lm_iterations_per_s"], d["ms_per_step"]))
PY
