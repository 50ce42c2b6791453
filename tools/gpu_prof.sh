# rocprofv3 kernel-trace --stats of the C4 bench and the C5-RS bench line
set -o pipefail
OUT=${1:-gpurun_out/prof}
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
cd /tmp && cd $ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4 -o c4 --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c4.json 2> $OUT/c4.err || { tail $OUT/c4.err; exit 1; }
python3 tools/iter_trace.py $OUT/c4/c4_kernel_trace.csv > $OUT/c4_iteration_trace.txt; rm -f $OUT/c4/c4_kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5rs -o c5rs --output-format csv -- python3 bench.py --config 4 --rolling-shutter 0.5 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/c5rs.json 2> $OUT/c5rs.err || { tail $OUT/c5rs.err; exit 1; }
rm -f $OUT/c5rs/c5rs_kernel_trace.csv
python3 tools/kstats.py $OUT/c4/c4_kernel_stats.csv > $OUT/c4_summary.txt
python3 tools/kstats.py $OUT/c5rs/c5rs_kernel_stats.csv > $OUT/c5rs_summary.txt
cat $OUT/c4_summary.txt | head -30; cat $OUT/c5rs_summary.txt | head -25
