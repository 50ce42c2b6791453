# Host-side timeline of the C4 iteration: rocprofv3 kernel trace + HIP runtime
# API trace (no counters) of a short bench run; tools/host_gap.py lines up
# each k_ne_bnd_jb launch call with the kernels around it.
set -o pipefail
OUT=${1:-gpurun_out/r5_host}
mkdir -p $OUT
cd /tmp && cd - > /dev/null
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $OUT/trace -o c4 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 tools/host_gap.py $OUT/trace > $OUT/host_gap.txt && cat $OUT/host_gap.txt
