# Round 3: backward record staging by global_load_lds (A/B) -- parity on each variant, then the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/glds; mkdir -p $O
for L in libgs_g1w4.so libgs_g1w6.so; do
GS_MI355X_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "backward_split or config1_parity or stale or graph_replay or edge" > $O/t_$L.log 2>&1
rc=$?; echo "$L tests rc=$rc"; tail -2 $O/t_$L.log; [ $rc -eq 0 ] || exit $rc
done
for L in libgs_mi355x.so libgs_g1w4.so libgs_g1w6.so libgs_mi355x.so libgs_g1w6.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); print('$L', round(d['ms_per_step'],4), 'bwd', round(d['stage_ms']['backward_blend'],4), 'fwd', round(d['stage_ms']['forward_blend'],4))"
done
