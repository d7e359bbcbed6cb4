# Blend-variant diagnosis: parity subsets of the default, the in-forward sort (fs) and the exp-window
# flags (ef); work counters (stats builds); bench A/B of the default, the quadrant forward at 8
# waves/SIMD (fq8), fs, the flagged forward exp (fx) and ef; SQ counters of the default and fq8.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
K="parity or depth_sort or bench_workload or graph"
echo "== tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K or sort" > gpurun_out/diag/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/diag/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/diag/pytest.log | head -20; exit $rc; }
for v in fs ef; do
  echo "== $v tests"; GS_MI355X_LIB=libgs_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/diag/pytest_$v.log 2>&1; rc=$?; tail -1 gpurun_out/diag/pytest_$v.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/diag/pytest_$v.log | head -20; exit $rc; }
done
for v in stats fqstats; do
  echo "== stats $v"; GS_MI355X_LIB=libgs_$v.so timeout -k 10 200 python scripts/blend_stats.py > gpurun_out/diag/stats_$v.log 2>&1 || { tail -5 gpurun_out/diag/stats_$v.log; exit 1; }
  head -3 gpurun_out/diag/stats_$v.log
done
echo "== ab"; VARIANTS="mi355x fq8 fs fx ef" REPS=2 STEPS=30 bash scripts/ab.sh || exit $?
echo "== sq"; VARIANTS="mi355x fq8" REPS=0 PMC="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_WAIT_ANY,SQ_BUSY_CYCLES" bash scripts/ab.sh > gpurun_out/diag/sq_ab.log 2>&1 || { tail -5 gpurun_out/diag/sq_ab.log; exit 1; }
echo diag-done
