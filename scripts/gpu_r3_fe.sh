# Round 3: the backward list split's front share (default 4/16; libgs_e1.so 3/16, libgs_e3.so 5/16;
# an earlier pass of this script: 1/8 and 3/8) with the XCD-group launch order: alternating bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fe; mkdir -p $O
for i in 1 2 3 4; do for L in libgs_mi355x.so libgs_e1.so libgs_e3.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), 'bwd', round(s['backward_blend'],4))"
done; done
