# kernel-trace profiles only (variants whose output may be wrong on purpose)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in ${VARIANTS:-mi355x}; do
  echo "== prof $v"
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof_$v -o p -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/rocprof_$v.log 2>&1 || { tail -5 gpurun_out/ab/rocprof_$v.log; exit 1; }
done
echo done
