# GPU-box A/B: parity tests + bench for each library variant named in $VARIANTS.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in ${VARIANTS:-mi355x}; do
  echo "== $v"
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/ab/pytest_$v.log 2>&1 || { tail -20 gpurun_out/ab/pytest_$v.log; exit 1; }
  tail -1 gpurun_out/ab/pytest_$v.log
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/bench_$v.log 2>&1 || { tail -5 gpurun_out/ab/bench_$v.log; exit 1; }
done
echo done
