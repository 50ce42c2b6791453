# A/B step of round 5: PCR probe variants, the K2 workgroup timeline, C2 and
# C5 bench lines.  usage: bash tools/gpu_ab.sh OUT
set -o pipefail
OUT=${1:?out}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in tools/ubench/pcr_probe_v*; do
  [ -x "$v" ] || continue
  timeout -k 10 60 "$v" > "$OUT/$(basename $v).txt" 2>&1 || { cat "$OUT/$(basename $v).txt"; exit 1; }
done
timeout -k 10 200 python -u bench.py --path probe=2 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > "$OUT/k2probe.json" 2> "$OUT/k2probe.err" || { tail "$OUT/k2probe.err"; exit 1; }
timeout -k 10 300 python -u bench.py --config 1 --steps 8 --warmup 3 --no-cpu-baseline --no-traffic > "$OUT/bench_1.json" 2> "$OUT/bench_1.err" || { tail "$OUT/bench_1.err"; exit 1; }
timeout -k 10 400 python -u bench.py --config 4 --steps 8 --warmup 3 --no-cpu-baseline > "$OUT/bench_4.json" 2> "$OUT/bench_4.err" || { tail "$OUT/bench_4.err"; exit 1; }
grep -h "best\|level" "$OUT"/pcr_probe_v*.txt
grep "mmba probe" "$OUT/k2probe.err"
echo done
