set -o pipefail
OUT=gpurun_out/r3a
mkdir -p $OUT
timeout -k 10 60 ./tools/ubench/bcr_item > $OUT/item.txt 2>&1 || exit 1
cat $OUT/item.txt
