# Round 3: u16 tile keys from the emission (working tree) vs libgs_base.so: GPU tests, alternating
# bench runs, config 5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/key16; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 1500 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for L in libgs_base.so libgs_mi355x.so libgs_base.so libgs_mi355x.so libgs_base.so libgs_mi355x.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), 'emit', round(s['pair_emit'],4), 'sort', round(s['tile_sort'],4), 'fwd', round(s['forward_blend'],4))"
done
for L in libgs_base.so libgs_mi355x.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench_configs.py --config 5 > $O/c5_$L.log 2>&1 || { tail -5 $O/c5_$L.log; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), {k: round(v,3) for k,v in s.items()})"
done
