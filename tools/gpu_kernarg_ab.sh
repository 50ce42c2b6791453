# HIP_FORCE_DEV_KERNARG A/B (kernel arguments in device memory) on C2 and C4, one box
set -o pipefail
OUT=${1:-gpurun_out/kernarg}
mkdir -p $OUT
for r in 1 2; do
  for v in 0 1; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python3 bench.py --config 1 --steps 12 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/c1_k${v}_$r.json 2> $OUT/c1_k${v}_$r.err || exit 1
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-traffic > $OUT/c4_k${v}_$r.json 2> $OUT/c4_k${v}_$r.err || exit 1
  done
done
python3 - $OUT <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    print("%-14s %8.0f LM it/s  device-resident %8.0f" % (f.split("/")[-1][:-5], d["lm_iterations_per_s"], d["device_resident"]["lm_iterations_per_s"]))
PY
