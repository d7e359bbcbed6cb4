# The whole -m gpu suite on the current library, then config 5 (fused step) and the bench, twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/suite; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "== tests: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit $rc; }
for r in 1 2; do
  timeout -k 10 400 python bench_configs.py --config 5 > $O/cfg5_$r.log 2>&1 || { tail -5 $O/cfg5_$r.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/cfg5_$r.log').read().strip().splitlines()[-1]); print('cfg5', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()})"
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$r.log 2>&1 || { tail -5 $O/bench_$r.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$r.log').read().strip().splitlines()[-1]); print('bench', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()})"
done
echo suite-done
