# The fused training-step backward (gs_backward_step) against the unfused sequence: the GPU tests
# that cover it, then config 5 (and the compacting-chain scene) timed both ways.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/step; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "fused or packed or chain_kernels or density_accumulate or adam or reached_tag" > $O/pytest.log 2>&1
rc=$?; echo "== tests: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit $rc; }
for r in 1 2; do
  for m in fused unfused; do
    timeout -k 10 400 python bench_configs.py --config 5 $( [ $m = unfused ] && echo --unfused ) > $O/cfg5_${m}_$r.log 2>&1 || { tail -5 $O/cfg5_${m}_$r.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/cfg5_${m}_$r.log').read().strip().splitlines()[-1]); print('$m', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()})"
  done
done
echo step-ab-done
