# SQ counters (one pass) for the hot per-observation kernels of one C4 solve.
set -o pipefail
OUT=${1:-gpurun_out/sq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-include-regex "k_jacobian_u|k_schur_dest_u|k_records|k_bcr_level|k_residual|k_schur_obs" -d $OUT/sq -o c4 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > $OUT/sq.json 2> $OUT/sq.err || exit 1
echo done
