# rocprofv3 kernel traces of C2 / C4 / C5 bench runs + one-iteration timelines
set -o pipefail
OUT=${1:-gpurun_out/iter}
mkdir -p $OUT
export TMPDIR=/tmp
for c in 1 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c$c -o c$c --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c$c.json 2> $OUT/c$c.err || { tail $OUT/c$c.err; exit 1; }
  python3 tools/iter_trace.py $OUT/c$c/c${c}_kernel_trace.csv > $OUT/c${c}_iteration.txt
  python3 tools/kstats.py $OUT/c$c/c${c}_kernel_stats.csv > $OUT/c${c}_summary.txt
  tail -1 $OUT/c${c}_iteration.txt
done
