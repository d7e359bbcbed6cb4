# Round 3: LSD tile sort with u16 keys between the passes and ranges from the last scatter (working
# tree) vs libgs_base.so: sort parity tests, then config 5 in alternating runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lsd16; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for L in libgs_base.so libgs_mi355x.so libgs_base.so libgs_mi355x.so; do
GS_MI355X_LIB=$L timeout -k 10 300 python bench_configs.py --config 5 > $O/c5_$L.log 2>&1 || { tail -5 $O/c5_$L.log; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_$L.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('$L', round(d['ms_per_step'],4), {k: round(v,3) for k,v in s.items()})"
done
timeout -k 10 1200 python -u -m pytest tests/test_gpu_full.py -m gpu -x -q --timeout 1500 --timeout-method thread -k "config5" > $O/t5.log 2>&1
rc=$?; tail -2 $O/t5.log; exit $rc
