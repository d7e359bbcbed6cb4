# Round 3: LSD tile-sort digit split A/B at config 5 + the sort parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lsd; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "tile_sort_paths or many_tiles or large_pair" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|^E " $O/tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
for L in libgs_mi355x.so libgs_lsd8.so libgs_mi355x.so libgs_lsd8.so; do
GS_MI355X_LIB=$L timeout -k 10 400 python bench_configs.py --config 5 > $O/c5_$L.log 2>&1 || { tail -5 $O/c5_$L.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/c5_$L.log').read().strip().splitlines()[-1]); print('$L', round(d['ms_per_step'],4), 'tile_sort', round(d['stage_ms']['tile_sort'],4))"
done
