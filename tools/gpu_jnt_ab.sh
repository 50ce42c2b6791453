# A/B: J rows stored non-temporal (tools/ab/libmmba_jnt.so, -DMMBA_J_NT) against the tree's build
set -o pipefail
OUT=${1:-gpurun_out/jnt}
mkdir -p $OUT
for r in 1 2 3; do
  for v in def jnt; do
    if [ $v = jnt ]; then export MMBA_LIB=$PWD/tools/ab/libmmba_jnt.so; else unset MMBA_LIB; fi
    timeout -k 10 300 python3 bench.py --config 1 --steps 12 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/c1_${v}_$r.json 2> $OUT/c1_${v}_$r.err || exit 1
    if [ $r -le 2 ]; then
      timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-traffic > $OUT/c4_${v}_$r.json 2> $OUT/c4_${v}_$r.err || exit 1
    fi
  done
done
unset MMBA_LIB
python3 - $OUT <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    print("%-12s %8.0f LM it/s  device-resident %8.0f  ms/solve %.3f" % (f.split("/")[-1][:-5], d["lm_iterations_per_s"], d["device_resident"]["lm_iterations_per_s"], d["ms_per_step"]))
PY
