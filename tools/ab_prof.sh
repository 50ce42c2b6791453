# A/B kernel stats: rocprofv3 --stats of one C4 bench step per env setting.
# usage: bash tools/ab_prof.sh <outdir> "ENV=a" "ENV=b" ...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for e in "$@"; do
  env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$i -o c4 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err || exit 1
  echo "$e" > $OUT/p$i/env.txt
  i=$((i+1))
done
echo done
