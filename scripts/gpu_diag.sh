# Diagnostic benches (no parity: the variants skip work on purpose) for each library in $VARIANTS.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in ${VARIANTS}; do
  echo "== $v"
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/bench_$v.log 2>&1 || { tail -5 gpurun_out/ab/bench_$v.log; exit 1; }
done
python scripts/ab_summary.py
