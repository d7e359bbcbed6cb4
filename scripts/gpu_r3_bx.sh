# Round 3: backward in the forward's XCD groups (libgs_bx.so, -DGS_BWD_XCD=1) vs the default build:
# parity subset with the variant, alternating bench runs, backward HBM reads of both
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/bx; mkdir -p $O
GS_MI355X_LIB=libgs_bx.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for L in libgs_mi355x.so libgs_bx.so libgs_mi355x.so libgs_bx.so libgs_mi355x.so libgs_bx.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), 'fwd', round(s['forward_blend'],4), 'bwd', round(s['backward_blend'],4))"
done
for L in libgs_mi355x.so libgs_bx.so; do
GS_MI355X_LIB=$L timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/f_$L -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 3 > /dev/null 2>&1 || exit 1
done
echo done
