# GPU-box check: smoke, GPU parity tests, one bench line, one rocprofv3 kernel-trace summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest"; SHOW=4 bash scripts/gpu_tests.sh || exit $?  # (-v -s: progress on the log; gpurun_out/pytest_gpu.log)
echo "== bench"; timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
echo "== rocprof"; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof.log 2>&1; rc=$?; tail -3 gpurun_out/rocprof.log; exit $rc
