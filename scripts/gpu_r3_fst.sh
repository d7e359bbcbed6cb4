# Round 3: the forward launch rank inside a bucket by tile order (ballots; libgs_fst.so) vs LDS atomics
# (default): parity subset with the variant, alternating bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fst; mkdir -p $O
GS_MI355X_LIB=libgs_fst.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3 4 5; do for L in libgs_mi355x.so libgs_fst.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > $O/b_$L.log 2>&1 || { tail -5 $O/b_$L.log; exit 1; }
python -c "import json; d=json.loads(open('$O/b_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), 'fwd', round(s['forward_blend'],4), 'bwd', round(s['backward_blend'],4))"
done; done
