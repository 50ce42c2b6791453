# C5 with the rolling shutter (configs[4] -rs 0.5): bench lines through two
# builds of libmmba.so (A/B, interleaved) and a kernel profile of the in-tree one.
#   gpurun -- 'bash tools/c5rs_ab.sh OUT tools/ab/libA.so mayamatchmovesolver_amd/csrc/libmmba.so'
set -o pipefail
OUT=${1:?out}; A=${2:?a}; B=${3:?b}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--config 4 --rolling-shutter 0.5 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic"
for r in 1 2; do
  for lib in "$A" "$B"; do
    tag=$(basename "$lib" .so)_r$r
    MMBA_LIB="$PWD/$lib" timeout -k 10 300 python -u bench.py $ARGS > "$OUT/c5rs_$tag.json" 2> "$OUT/c5rs_$tag.err" || { tail "$OUT/c5rs_$tag.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['lm_iterations_per_s'],1), 'it/s', round(d['ms_per_step'],3), 'ms/step')" "$OUT/c5rs_$tag.json" "$tag"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c5rs --output-format csv -- python3 bench.py --config 4 --rolling-shutter 0.5 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > "$OUT/prof.json" 2> "$OUT/prof.err" || { tail "$OUT/prof.err"; exit 1; }
rm -f "$OUT/prof/c5rs_kernel_trace.csv"
python3 - "$OUT/prof/c5rs_kernel_stats.csv" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
for x in r[:12]:
    print(x["Name"][:60].ljust(60), x["Calls"], round(float(x["AverageNs"]) / 1000, 2), x["Percentage"][:5])
PY
echo "c5rs done"
