# Per-frame solve mode throughput on C2 (120 frames): 1, 4 and 16 frames in flight.
set -o pipefail
OUT=${1:-gpurun_out/perframe}
mkdir -p $OUT
for c in 1 4 16; do
  timeout -k 10 300 python -u bench.py --config 1 --per-frame $c --steps 2 --warmup 1 > $OUT/pf_$c.json 2> $OUT/pf_$c.err || exit 1
done
echo "all done"
