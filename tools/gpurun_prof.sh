set -o pipefail
mkdir -p gpurun_out/prof_r1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o c4 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r1/bench.json 2> gpurun_out/prof_r1/bench.err
echo "exit=$?" >> gpurun_out/prof_r1/bench.err
find gpurun_out/prof_r1 -name "*stats*" | head
