# Round 3: quick GPU check of selected tests: bash scripts/gpu_r3_quick.sh "<pytest -k expr>" [files...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3q
K="$1"; shift
FILES="${@:-tests}"
timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v -s --timeout 600 --timeout-method thread -k "$K" > gpurun_out/r3q/quick.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|^E " gpurun_out/r3q/quick.log | tail -40
exit $rc
