# Round-5 first GPU call: the N>1 launcher rehearsal, the -m gpu suite, then the quadrant-group
# forward variant (libgs_fq.so) on the parity subset and A/B against the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== dist"; bash scripts/gpu_dist_rehearsal.sh || exit $?
echo "== tests"; SHOW=6 bash scripts/gpu_tests.sh || exit $?
echo "== fq tests"; GS_MI355X_LIB=libgs_fq.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or bench_workload or config4 or general_camera" > gpurun_out/pytest_fq.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_fq.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_fq.log | head -20; exit $rc; }
echo "== ab"; VARIANTS="mi355x fq" REPS=3 STEPS=30 bash scripts/ab.sh || exit $?
