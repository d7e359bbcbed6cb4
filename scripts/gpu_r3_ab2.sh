# Round 3: A/B of the working tree (libgs_mi355x.so) against libgs_base.so: parity subset, then
# alternating bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for L in libgs_base.so libgs_mi355x.so libgs_base.so libgs_mi355x.so libgs_base.so libgs_mi355x.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), 'fwd', round(s['forward_blend'],4), 'bwd', round(s['backward_blend'],4), 'chain', round(s['chain'],4))"
done
