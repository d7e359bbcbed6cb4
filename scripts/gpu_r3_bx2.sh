# Round 3: backward in the forward's XCD groups as the default (working tree) vs -DGS_BWD_XCD=0
# (libgs_nobx.so): full GPU suite, then alternating bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/bx2; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 1500 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3 4 5; do for L in libgs_nobx.so libgs_mi355x.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), 'fwd', round(s['forward_blend'],4), 'bwd', round(s['backward_blend'],4))"
done; done
