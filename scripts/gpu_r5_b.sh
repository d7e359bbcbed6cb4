# Quadrant-forward diagnosis: work counters (stats builds), then SQ counter passes + kernel stats of
# the default and the quadrant forward; parity subset of the default (sort-kernel LDS padding).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
echo "== tests"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or depth_sort or sort" > gpurun_out/diag/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/diag/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/diag/pytest.log | head -20; exit $rc; }
for v in stats fqstats; do
  echo "== stats $v"; GS_MI355X_LIB=libgs_$v.so timeout -k 10 200 python scripts/blend_stats.py > gpurun_out/diag/stats_$v.log 2>&1 || { tail -5 gpurun_out/diag/stats_$v.log; exit 1; }
  head -3 gpurun_out/diag/stats_$v.log
done
echo "== ab"; VARIANTS="mi355x fq" REPS=2 STEPS=30 PROF=1 PMC="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_WAIT_ANY,SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_INSTS_VMEM" bash scripts/ab.sh || exit $?
