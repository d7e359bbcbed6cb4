# Round 3: chain compaction A/B (bench + config 5) with a parity subset on the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/chain; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "backward_split or config1_parity or stale or graph_replay or edge or packed or split_backward or bench_workload" > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for L in libgs_chold.so libgs_mi355x.so libgs_cp2.so libgs_chold.so libgs_mi355x.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); print('$L', round(d['ms_per_step'],4), 'chain', round(d['stage_ms']['chain'],4))"
GS_MI355X_LIB=$L timeout -k 10 400 python bench_configs.py --config 5 > $O/c5_$L.log 2>&1 || { tail -5 $O/c5_$L.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/c5_$L.log').read().strip().splitlines()[-1]); print('  cfg5', round(d['ms_per_step'],4), 'chain', round(d['stage_ms']['chain'],4))"
done
