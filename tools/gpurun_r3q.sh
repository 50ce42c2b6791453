set -o pipefail
OUT=gpurun_out/r3q
mkdir -p $OUT
MMBA_PROBE=1 timeout -k 10 120 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/probe.json 2> $OUT/probe.err || exit 1
grep "mmba probe" $OUT/probe.err
