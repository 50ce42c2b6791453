set -o pipefail
OUT=gpurun_out/r3m
mkdir -p $OUT
for pw in 6 12 24; do
timeout -k 10 60 ./tools/ubench/bcr_item_pw$pw > $OUT/item_pw$pw.txt 2>&1 || exit 1
echo "PW=$pw"; grep -A1 "run 2" $OUT/item_pw$pw.txt
done
