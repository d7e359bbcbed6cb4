# One parametrised GPU-box A/B driver (replaces the round-3 one-off gpu_r3_*.sh scripts).
#   VARIANTS="mi355x foo"  library variants (gaussiansplatting_amd/lib/libgs_<v>.so; build_variant.sh)
#   REPS=2                 alternating bench runs per variant
#   TESTS=1                run the -m gpu suite on every variant first (PYTEST_K narrows it; TESTV:
#                          only on these variants)
#   STEPS=30 BENCH_ARGS=   extra bench.py arguments (e.g. --gaussians 5000000)
#   CFG=5                  also run bench_configs.py --config $CFG per variant
#   PROF=1                 rocprofv3 kernel-trace stats per variant
#   PMC="FETCH_SIZE WRITE_SIZE"  one rocprofv3 --pmc pass per counter group per variant
# Output under gpurun_out/ab/, summary on stdout.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
[ "${REPS:-2}" -gt 0 ] && rm -f $O/bench_*.log
for v in ${TESTV:-${VARIANTS:-mi355x}}; do
  if [ -n "$TESTS" ]; then
    GS_MI355X_LIB=libgs_$v.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_$v.log 2>&1
    rc=$?; echo "== tests $v: $(tail -1 $O/pytest_$v.log)"; [ $rc -eq 0 ] || { tail -30 $O/pytest_$v.log; exit $rc; }
  fi
done
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-mi355x}; do
    GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline $BENCH_ARGS > $O/bench_${v}_$r.log 2>&1 || { tail -5 $O/bench_${v}_$r.log; exit 1; }
    if [ -n "$CFG" ]; then
      GS_MI355X_LIB=libgs_$v.so timeout -k 10 400 python bench_configs.py --config $CFG > $O/cfg${CFG}_${v}_$r.log 2>&1 || { tail -5 $O/cfg${CFG}_${v}_$r.log; exit 1; }
    fi
  done
done
for v in ${VARIANTS:-mi355x}; do
  if [ -n "$PROF" ]; then
    GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python bench.py --no-cpu-baseline --steps 10 --warmup 5 $BENCH_ARGS > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  fi
  for c in $PMC; do
    GS_MI355X_LIB=libgs_$v.so timeout -s KILL 120 rocprofv3 --pmc ${c//,/ } --kernel-trace --output-format csv -d $O/pmc_${v}_${c//,/_} -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 3 $BENCH_ARGS > $O/pmc_${v}.log 2>&1 || { tail -5 $O/pmc_${v}.log; exit 1; }
  done
done
python scripts/ab_summary.py
echo ab-done
