# GPU-box steps, run through gpurun from the repo root:
#   gpurun --timeout 1200 -- 'bash tools/gpu.sh OUT STEP [STEP ...]'
# Steps (each under its own time limit; the first failure ends the call):
#   tests[:PYTEST_K]  the -m gpu suite (optionally only tests matching -k)
#   testsall          the -m gpu suite without -x (every failure in one call)
#   smoke             __graft_entry__.smoke()
#   bench             the default bench line (C4, CPU baseline, PMC traffic)
#   benchcfg:I        bench line of configs[I] (no CPU baseline)
#   benchpath:N=V     default-config bench line with a pinned path (--path N=V)
#   benchlib:FILE     default-config bench line (C4, 8 steps) through another build of libmmba.so (MMBA_LIB)
#   prof              rocprofv3 --kernel-trace --stats of the default bench
#   pmc               FETCH_SIZE / WRITE_SIZE passes of the default bench
#   sqpmc             one pass of 8 SQ counters (wave cycles, waits, VALU) on the default bench
#   cfgpmc:I          FETCH_SIZE / WRITE_SIZE / SQ passes of configs[I]
#   iter              kernel traces + one-iteration timelines of C2 / C4 / C5
#   ubench            tools/ubench dgemm_probe (C3 update shapes) and pcr_probe (C4 system)
set -o pipefail
OUT=${1:?out dir}
shift
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
for step in "$@"; do
  case "$step" in
    testsall)
      # every failure in one call; the steps after it still run unless the
      # run faulted or timed out (pytest: 1 = failed tests, 2+ = other)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
      rc=$?; tail -40 "$OUT/tests.log"; [ $rc -le 1 ] || exit $rc ;;
    tests*)
      K=${step#tests}; K=${K#:}
      if [ -n "$K" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$K" > "$OUT/tests.log" 2>&1
      else
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
      fi
      rc=$?; tail -25 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; } ;;
    bench)
      timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    benchcfg:*)
      c=${step#benchcfg:}
      st=8; wu=3
      if [ "$c" = 2 ]; then st=3; wu=1; fi  # C3: ~11 s per solve
      cb=--no-cpu-baseline
      if [ "$c" = 1 ] || [ "$c" = 4 ]; then cb=; fi  # C2 / C5: the CPU windows + the full-config oracle run
      timeout -k 10 600 python -u bench.py --config "$c" --steps $st --warmup $wu $cb --no-traffic > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { tail "$OUT/bench_$c.err"; exit 1; }
      cat "$OUT/bench_$c.json" ;;
    benchpath:*)
      pv=${step#benchpath:}
      timeout -k 10 400 python -u bench.py --path "$pv" --steps 8 --warmup 3 --no-cpu-baseline --no-traffic > "$OUT/bench_$pv.json" 2> "$OUT/bench_$pv.err" || { tail "$OUT/bench_$pv.err"; exit 1; }
      cat "$OUT/bench_$pv.json" ;;
    benchlib:*)
      lib=${step#benchlib:}; tag=$(basename "$lib" .so)
      MMBA_LIB="$ROOT/$lib" timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-traffic > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail "$OUT/bench_$tag.err"; exit 1; }
      cat "$OUT/bench_$tag.json" ;;
    prof)
      cd /tmp && cd "$ROOT"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c4 --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { tail "$OUT/prof_bench.err"; exit 1; }
      python3 tools/iter_trace.py "$OUT/prof/c4_kernel_trace.csv" > "$OUT/c4_iteration_trace.txt" && rm -f "$OUT/prof/c4_kernel_trace.csv" ;;
    pmc)
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$OUT/pmc_$ctr" -o c4 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > "$OUT/pmc_$ctr.json" 2> "$OUT/pmc_$ctr.err" || exit 1
      done ;;
    sqpmc)
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d "$OUT/sqpmc" -o c4 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > "$OUT/sqpmc.json" 2> "$OUT/sqpmc.err" || { tail "$OUT/sqpmc.err"; exit 1; }
      python3 tools/pmc_summary.py "$OUT/sqpmc" > "$OUT/sqpmc_summary.txt" && cat "$OUT/sqpmc_summary.txt" ;;
    cfgpmc:*)
      # FETCH_SIZE, WRITE_SIZE and the SQ pass on configs[I] (one solve each)
      c=${step#cfgpmc:}
      for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"; do
        tag=${ctr%% *}
        timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$OUT/c${c}_$tag" -o c$c --output-format csv -- python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-traffic > "$OUT/c${c}_$tag.json" 2> "$OUT/c${c}_$tag.err" || { tail "$OUT/c${c}_$tag.err"; exit 1; }
        python3 tools/pmc_summary.py "$OUT/c${c}_$tag" > "$OUT/c${c}_${tag}_summary.txt" && head -14 "$OUT/c${c}_${tag}_summary.txt"
      done ;;
    ubench)
      timeout -k 10 120 tools/ubench/dgemm_probe > "$OUT/dgemm_probe.txt" 2>&1 || { cat "$OUT/dgemm_probe.txt"; exit 1; }
      timeout -k 10 120 tools/ubench/pcr_probe > "$OUT/pcr_probe.txt" 2>&1 || { cat "$OUT/pcr_probe.txt"; exit 1; }
      cat "$OUT/dgemm_probe.txt" "$OUT/pcr_probe.txt" ;;
    iter)
      bash tools/gpu_iter.sh "$OUT/iter" || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
