# GPU test cycle: the -m gpu suite (one process), optional extra pytest args.
# usage: bash tools/gpurun_tests.sh <outdir> [pytest selection...]
set -o pipefail
OUT=${1:-gpurun_out/tests}
shift
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -q --maxfail=${MAXFAIL:-1} --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -30 $OUT/tests.log
exit $rc
