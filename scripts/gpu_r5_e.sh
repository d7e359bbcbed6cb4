# Quadrant forward (now the default) against its list-index prefetch at 8 (fqp, 5 spilled VGPRs) and
# 7 waves/SIMD (fqpu), and against the band forward (band); the default's -m gpu suite first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== tests"; SHOW=4 bash scripts/gpu_tests.sh || exit $?
mkdir -p gpurun_out/diag
K="parity or depth_sort or bench_workload or graph"
for v in fqp; do
  echo "== $v tests"; GS_MI355X_LIB=libgs_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/diag/pytest_$v.log 2>&1; rc=$?; tail -1 gpurun_out/diag/pytest_$v.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/diag/pytest_$v.log | head -20; exit $rc; }
done
echo "== ab"; VARIANTS="mi355x fqp fqpu band" REPS=2 STEPS=30 bash scripts/ab.sh || exit $?
