# RCCL rehearsal: 2 ranks (one process each) on the box's one GPU, the driver's
# multi-GPU launch command with MMBA_BENCH_DEVICE=0; small scene, then the full
# weak-scaling shard (2 x C4); timings are not scaling numbers (one GPU shared)
set -o pipefail
OUT=gpurun_out/r3j
mkdir -p $OUT
NCCL_DEBUG=WARN MMBA_BENCH_DEVICE=0 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config 3 --frames 40 --scale 0.2 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/n2_small.json 2> $OUT/n2_small.err || { tail -20 $OUT/n2_small.err; exit 1; }
cat $OUT/n2_small.json
NCCL_DEBUG=WARN MMBA_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/n2_c4.json 2> $OUT/n2_c4.err || { tail -20 $OUT/n2_c4.err; exit 1; }
cat $OUT/n2_c4.json
echo done
