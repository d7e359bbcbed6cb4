# Config-5 A/B of library variants (gaussiansplatting_amd/lib/libgs_<v>.so, scripts/build_variant.sh):
#   VARIANTS="mi355x foo"  REPS=2 alternating bench_configs.py --config 5 runs per variant
#   TESTS=1 PYTEST_K=...   the -m gpu tests on every variant first (TESTV: only on these variants)
#   ARGS=                  extra bench_configs.py arguments (e.g. --depth-sort 2)
# plus one rocprofv3 kernel trace per variant; summary (step times, per-frame kernel times) on stdout.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab5; mkdir -p $O; rm -rf $O/*
for v in ${TESTV:-${VARIANTS:-mi355x}}; do
  if [ -n "$TESTS" ]; then
    GS_MI355X_LIB=libgs_$v.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_$v.log 2>&1
    rc=$?; echo "== tests $v: $(tail -1 $O/pytest_$v.log)"; [ $rc -eq 0 ] || { tail -30 $O/pytest_$v.log; exit $rc; }
  fi
done
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-mi355x}; do
    GS_MI355X_LIB=libgs_$v.so timeout -k 10 400 python bench_configs.py --config 5 $ARGS > $O/cfg5_${v}_$r.log 2>&1 || { tail -5 $O/cfg5_${v}_$r.log; exit 1; }
  done
done
for v in ${VARIANTS:-mi355x}; do
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$v -o run -- python bench_configs.py --config 5 --steps 5 --warmup 2 $ARGS > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
done
python scripts/ab5_summary.py $O ${VARIANTS:-mi355x}
echo ab5-done
