set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag
GS_MI355X_LIB=libgs_stats.so timeout -k 10 300 python scripts/blend_stats.py > gpurun_out/diag/stats.log 2>&1 || { tail -20 gpurun_out/diag/stats.log; exit 1; }
cat gpurun_out/diag/stats.log
GS_MI355X_LIB=libgs_btrace.so timeout -k 10 300 python scripts/blend_trace.py > gpurun_out/diag/trace.log 2>&1 || { tail -20 gpurun_out/diag/trace.log; exit 1; }
cat gpurun_out/diag/trace.log
