set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg5prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfg5prof -o p -- python bench_configs.py --config 5 --steps 3 --warmup 2 > gpurun_out/cfg5prof/log 2>&1 || { tail -5 gpurun_out/cfg5prof/log; exit 1; }
echo ok
