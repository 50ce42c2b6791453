set -o pipefail
OUT=gpurun_out/r5_occ
mkdir -p $OUT
cd tools/ubench
timeout -k 10 60 ./pcr_probe 2994 2 > ../../$OUT/probe_2994_2.txt 2>&1 || exit 1

timeout -k 10 60 ./pcr_probe 5988 2 > ../../$OUT/probe_5988_2.txt 2>&1 || exit 1

cd ../..
cat $OUT/probe_*.txt
timeout -k 10 400 python -u tools/big_band.py 1 2 4 8 > $OUT/big_band.txt 2>&1 || { cat $OUT/big_band.txt; exit 1; }
cat $OUT/big_band.txt
