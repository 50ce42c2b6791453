# RCCL rehearsal: 2 ranks on the one GPU of the box (weak-scaling bench path)
set -o pipefail
OUT=gpurun_out/rccl
mkdir -p $OUT
NCCL_DEBUG=WARN MMBA_BENCH_DEVICE=0 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config 3 --frames 40 --scale 0.2 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/n2.json 2> $OUT/n2.err
rc=$?
tail -5 $OUT/n2.err
cat $OUT/n2.json
exit $rc
