# A/B benches on the GPU box: bash tools/gpu_ab.sh OUT "PYTEST_K" [ENV=VAL ...]
# Runs the -m gpu tests matching PYTEST_K with the extra environment, then
# C4 and C2 bench lines with and without it (8 steps, 3 warmup).
set -o pipefail
OUT=${1:?out}; K=${2:?pytest -k}; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$K" != "-" ]; then
  env "$@" timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
  tail -2 "$OUT/tests.log"
fi
for c in 3 1; do
  env "$@" timeout -k 10 300 python bench.py --config $c --steps 8 --warmup 3 --no-cpu-baseline --no-traffic > "$OUT/c${c}_B.json" 2> "$OUT/c${c}_B.err" || { tail "$OUT/c${c}_B.err"; exit 1; }
  timeout -k 10 300 python bench.py --config $c --steps 8 --warmup 3 --no-cpu-baseline --no-traffic > "$OUT/c${c}_A.json" 2> "$OUT/c${c}_A.err" || { tail "$OUT/c${c}_A.err"; exit 1; }
done
python3 - "$OUT" <<'PY'
import json, sys
o = sys.argv[1]
for c in (3, 1):
    for v in ("A", "B"):
        d = json.load(open(f"{o}/c{c}_{v}.json"))
        print(c, v, d["config"]["workload"], round(d["ms_per_step"], 4), round(d["lm_iterations_per_s"], 1))
PY
