# One bench line under an environment: bash tools/gpu_bench_env.sh OUT NAME CONFIG [ENV=VAL ...]
set -o pipefail
OUT=${1:?out}; NAME=${2:?name}; C=${3:?config}; shift 3
mkdir -p "$OUT"
env "$@" timeout -k 10 300 python bench.py --config "$C" --steps 8 --warmup 3 --no-cpu-baseline --no-traffic > "$OUT/$NAME.json" 2> "$OUT/$NAME.err" || { tail "$OUT/$NAME.err"; exit 1; }
python3 -c "import json,sys; d=json.load(open('$OUT/$NAME.json')); print('$NAME', d['config']['workload'], round(d['ms_per_step'],4), round(d['lm_iterations_per_s'],1))"
