# Round 3: the per-tile work added to the list length when the XCD runs are cut (default 16;
# libgs_e1.so 0, libgs_e3.so 64): alternating bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tw; mkdir -p $O
for i in 1 2 3 4; do for L in libgs_mi355x.so libgs_e1.so libgs_e3.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), 'fwd', round(s['forward_blend'],4), 'bwd', round(s['backward_blend'],4))"
done; done
