set -o pipefail
OUT=gpurun_out/r6_c2
mkdir -p $OUT
for r in 1 2; do
timeout -k 10 300 python3 bench.py --config 1 --no-cpu-baseline --no-traffic > $OUT/split_$r.json 2>$OUT/split_$r.err || exit 1
timeout -k 10 300 python3 bench.py --config 1 --no-cpu-baseline --no-traffic --path NE_CF_SPLIT=0 > $OUT/nosplit_$r.json 2>$OUT/nosplit_$r.err || exit 1
done
bash tools/gpu_iter.sh $OUT/iter
