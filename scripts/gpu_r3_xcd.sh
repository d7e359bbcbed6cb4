# Round 3 experiment: XCD-aware forward launch order (host-computed, eager steps) vs the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/xcd; mkdir -p $O
for L in libgs_mi355x.so libgs_xw16.so libgs_xw64.so libgs_mi355x.so libgs_xw16.so libgs_xw64.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 20 > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), 'fwd', round(s['forward_blend'],4), 'bwd', round(s['backward_blend'],4))"
done
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/f1 -o run -- python bench.py --no-cpu-baseline --no-graph --steps 3 --warmup 2 > /dev/null 2>&1 || exit 1
GS_MI355X_LIB=libgs_xw16.so timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/f2 -o run -- python bench.py --no-cpu-baseline --no-graph --steps 3 --warmup 2 > /dev/null 2>&1 || exit 1
echo done
