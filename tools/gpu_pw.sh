# PCR probe at pivot-chain panel widths 4 / 6 (the build's) / 8 / 12
set -o pipefail
OUT=${1:-gpurun_out/r5_pw}
mkdir -p $OUT
cd tools/ubench
for v in pcr_probe_old pcr_probe pcr_probe_pw4 pcr_probe_pw8 pcr_probe_pw12 pcr_probe_old pcr_probe; do
  timeout -k 10 60 ./$v 2994 > ../../$OUT/$v.txt 2>&1 || { cat ../../$OUT/$v.txt; exit 1; }
  echo "$v: $(grep best ../../$OUT/$v.txt | head -1)"
done
