# Blend-variant diagnosis: parity subsets of the default and the in-forward sort (libgs_fs.so), work
# counters (stats builds), then bench A/B + kernel stats + SQ counter passes of the default, the
# quadrant forward at 8 waves/SIMD (fq8) and the in-forward sort (fs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
echo "== tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or depth_sort or sort" > gpurun_out/diag/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/diag/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/diag/pytest.log | head -20; exit $rc; }
echo "== fs tests"; GS_MI355X_LIB=libgs_fs.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or depth_sort or bench_workload or graph" > gpurun_out/diag/pytest_fs.log 2>&1; rc=$?; tail -2 gpurun_out/diag/pytest_fs.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/diag/pytest_fs.log | head -20; exit $rc; }
for v in stats fqstats; do
  echo "== stats $v"; GS_MI355X_LIB=libgs_$v.so timeout -k 10 200 python scripts/blend_stats.py > gpurun_out/diag/stats_$v.log 2>&1 || { tail -5 gpurun_out/diag/stats_$v.log; exit 1; }
  head -3 gpurun_out/diag/stats_$v.log
done
echo "== ab"; VARIANTS="mi355x fq8 fs" REPS=2 STEPS=30 PROF=1 PMC="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_WAIT_ANY,SQ_BUSY_CYCLES" bash scripts/ab.sh || exit $?
