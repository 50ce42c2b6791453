# C2 hand-back A/B on one box: default (speculative host-mapped hand-back),
# no speculation, DMA copies; alternating, 2 rounds each
set -o pipefail
OUT=${1:-gpurun_out/c2hb}
mkdir -p $OUT
for r in 1 2; do
  for v in def PRE_HANDBACK=0 HANDBACK_DMA=1 NE_CF_SPLIT=0; do
    a=; [ $v = def ] || a="--path $v"
    timeout -k 10 300 python3 bench.py --config 1 --steps 12 --warmup 3 --no-cpu-baseline --no-traffic $a > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit 1
  done
done
python3 - $OUT <<'PY'
import json, glob, sys, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f)); k = f.split("/")[-1].rsplit("_", 1)[0]
    acc[k].append((d["lm_iterations_per_s"], d["device_resident"]["lm_iterations_per_s"]))
for k, v in acc.items():
    print("%-16s handed-back %s   device-resident %s" % (k, " ".join("%.0f" % a for a, _ in v), " ".join("%.0f" % b for _, b in v)))
PY
