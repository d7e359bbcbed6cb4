# GPU-box A/B: parity tests of $TESTED variants, kernel-trace profile + bench of every variant in $VARIANTS.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in ${TESTED:-mi355x}; do
  echo "== test $v"
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/ab/pytest_$v.log 2>&1 || { tail -20 gpurun_out/ab/pytest_$v.log; exit 1; }
  tail -1 gpurun_out/ab/pytest_$v.log
done
for v in ${VARIANTS:-mi355x}; do
  echo "== bench $v"
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/bench_$v.log 2>&1 || { tail -5 gpurun_out/ab/bench_$v.log; exit 1; }
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof_$v -o p -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/rocprof_$v.log 2>&1 || { tail -5 gpurun_out/ab/rocprof_$v.log; exit 1; }
done
echo done
