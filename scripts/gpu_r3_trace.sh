set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3t
for s in 0 -1 4096; do
  GS_MI355X_LIB=libgs_btrace.so timeout -k 10 200 python scripts/blend_trace2.py $s > gpurun_out/r3t/trace_$s.txt 2>&1 || { tail -5 gpurun_out/r3t/trace_$s.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r3t/trace_$s.txt
done
