# GPU box: the -m gpu suite, then the bench (and the blend work counters if libgs_stats.so exists).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/ab/pytest.log 2>&1 || { tail -40 gpurun_out/ab/pytest.log; exit 1; }
tail -n 2 gpurun_out/ab/pytest.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab/bench_mi355x.log 2>&1 || { tail -5 gpurun_out/ab/bench_mi355x.log; exit 1; }
python scripts/ab_summary.py
if [ -f gaussiansplatting_amd/lib/libgs_stats.so ]; then
  GS_MI355X_LIB=libgs_stats.so timeout -k 10 300 python scripts/blend_stats.py > gpurun_out/ab/stats.log 2>&1 || { tail -5 gpurun_out/ab/stats.log; exit 1; }
  cat gpurun_out/ab/stats.log
fi
