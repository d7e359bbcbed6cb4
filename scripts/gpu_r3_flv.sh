# Round 3: forward launch-order levels per doubling of the list length inside an XCD group
# (default 2.5; libgs_f20.so 2.0, libgs_f30.so 3.0): alternating bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/flv; mkdir -p $O
for i in 1 2 3 4; do for L in libgs_mi355x.so libgs_f20.so libgs_f30.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), 'fwd', round(s['forward_blend'],4), 'bwd', round(s['backward_blend'],4))"
done; done
