# Quadrant forward v2 (scalar math, shared quadrant cull, in-forward sort) at 8 waves/SIMD (fq9, 2
# spilled VGPRs) and unbounded (fq9u, 70 VGPRs): parity subset, then A/B against the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
K="parity or depth_sort or bench_workload or graph"
for v in fq9; do
  echo "== $v tests"; GS_MI355X_LIB=libgs_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/diag/pytest_$v.log 2>&1; rc=$?; tail -1 gpurun_out/diag/pytest_$v.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/diag/pytest_$v.log | head -20; exit $rc; }
done
echo "== ab"; VARIANTS="mi355x fq9 fq9u" REPS=3 STEPS=30 bash scripts/ab.sh || exit $?
