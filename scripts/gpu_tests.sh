# GPU-box test run with progress on the log (every test's name as it starts, the tests' own notes):
#   PYTEST_K="expr" bash scripts/gpu_tests.sh      (all -m gpu tests without PYTEST_K)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${TESTS_TIMEOUT:-1100} python -u -m pytest tests -m gpu -x -v -s --timeout ${TEST_TIMEOUT:-300} \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -${SHOW:-40}
exit $rc
