# The long lists in one launch (tile_long_sort_kernel, workgroup MSD split) under the in-forward sort:
# the depth-order tests, the bench line, configs 2 and 5 in per-tile mode, the work counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/diag gpurun_out/cfg
echo "== tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or depth_sort or sort or bench_workload or graph or config5" > gpurun_out/diag/pytest_f.log 2>&1; rc=$?; tail -1 gpurun_out/diag/pytest_f.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/diag/pytest_f.log | head -20; exit $rc; }
echo "== bench"; timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_f.log 2>&1 || { tail -5 gpurun_out/bench_f.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_f.log').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()})"
for a in "2 2" "5 2"; do set -- $a
  timeout -k 10 400 python bench_configs.py --config $1 --depth-sort $2 > gpurun_out/cfg/cfg$1_d$2.log 2>&1 || { tail -5 gpurun_out/cfg/cfg$1_d$2.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/cfg/cfg$1_d$2.log').read().strip().splitlines()[-1]); print('cfg$1 d$2', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()})"
done
echo "== stats"; GS_MI355X_LIB=libgs_stats.so timeout -k 10 200 python scripts/blend_stats.py > gpurun_out/diag/stats_q.log 2>&1 || { tail -5 gpurun_out/diag/stats_q.log; exit 1; }
head -6 gpurun_out/diag/stats_q.log
