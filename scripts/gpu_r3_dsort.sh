# Round 3: depth sort in 3 passes of 11-bit digits (working tree) vs 8-bit digits (libgs_d8.so) and HEAD (libgs_base.so)
# at the bench workload (alternating runs, kernel stats) and at config 5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ds; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for L in libgs_base.so libgs_mi355x.so libgs_d8.so libgs_base.so libgs_mi355x.so libgs_d8.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), 'fwd', round(s['forward_blend'],4), 'bwd', round(s['backward_blend'],4), 'dsort', round(s['depth_sort'],4), 'proj', round(s['project'],4))"
done
for L in libgs_base.so libgs_mi355x.so; do
GS_MI355X_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$L -o run -- python bench.py --no-cpu-baseline --steps 10 --warmup 5 > /dev/null 2>&1 || exit 1
done
for L in libgs_base.so libgs_mi355x.so libgs_base.so libgs_mi355x.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench_configs.py --config 5 > $O/c5_$L.log 2>&1 || { tail -5 $O/c5_$L.log; exit 1; }
echo c5 $L; tail -1 $O/c5_$L.log | cut -c1-400
done
echo done
