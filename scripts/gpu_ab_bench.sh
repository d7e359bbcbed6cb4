# GPU-box A/B, timing only (variants that change scheduling, not results): bench for each library
# variant named in $VARIANTS, then the per-stage summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/bench_*.log
for v in ${VARIANTS:-mi355x}; do
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline > gpurun_out/ab/bench_$v.log 2>&1 || { tail -5 gpurun_out/ab/bench_$v.log; exit 1; }
done
python scripts/ab_summary.py
