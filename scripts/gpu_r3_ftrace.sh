set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3t
GS_MI355X_LIB=libgs_btrace.so timeout -k 10 200 python scripts/fwd_trace.py > gpurun_out/r3t/ftrace.txt 2>&1 || { tail -5 gpurun_out/r3t/ftrace.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r3t/ftrace.txt
GS_MI355X_LIB=libgs_btrace.so timeout -k 10 200 python scripts/blend_trace2.py -1 > gpurun_out/r3t/btrace.txt 2>&1 || { tail -5 gpurun_out/r3t/btrace.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r3t/btrace.txt
