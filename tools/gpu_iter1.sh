# rocprofv3 kernel trace of one config's bench run + its one-iteration timeline
#   bash tools/gpu_iter1.sh OUT CONFIG [bench args...]
set -o pipefail
OUT=${1:?out}; c=${2:?config}; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c$c -o c$c --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-traffic "$@" > $OUT/c$c.json 2> $OUT/c$c.err || { tail $OUT/c$c.err; exit 1; }
python3 tools/iter_trace.py $OUT/c$c/c${c}_kernel_trace.csv > $OUT/c${c}_iteration.txt
python3 tools/kstats.py $OUT/c$c/c${c}_kernel_stats.csv > $OUT/c${c}_summary.txt
cat $OUT/c${c}_iteration.txt; head -16 $OUT/c${c}_summary.txt
