set -o pipefail
OUT=gpurun_out/r2y
mkdir -p $OUT
timeout -k 10 60 ./tools/ubench/bcr_chain > $OUT/chain.txt 2>&1 || exit 1
cat $OUT/chain.txt
