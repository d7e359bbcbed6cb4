# Config-2 A/B of library variants (gaussiansplatting_amd/lib/libgs_<v>.so, scripts/build_variant.sh):
#   VARIANTS="mi355x foo" REPS=3 TESTS=1 TESTV=... PYTEST_K=...   (as scripts/ab_cfg5.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab2; mkdir -p $O; rm -rf $O/*
for v in ${TESTV:-${VARIANTS:-mi355x}}; do
  if [ -n "$TESTS" ]; then
    GS_MI355X_LIB=libgs_$v.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_$v.log 2>&1
    rc=$?; echo "== tests $v: $(tail -1 $O/pytest_$v.log)"; [ $rc -eq 0 ] || { tail -30 $O/pytest_$v.log; exit $rc; }
  fi
done
for r in $(seq 1 ${REPS:-3}); do
  for v in ${VARIANTS:-mi355x}; do
    GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 python bench_configs.py --config 2 $ARGS > $O/cfg2_${v}_$r.log 2>&1 || { tail -5 $O/cfg2_${v}_$r.log; exit 1; }
    python -c "import json;d=json.loads(open('$O/cfg2_${v}_$r.log').read().strip().splitlines()[-1]);print('$v',$r,round(d['ms_per_step'],4),{k:round(x,4) for k,x in d['stage_ms'].items() if x})"
  done
done
echo ab2-done
