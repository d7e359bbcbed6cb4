# Config 5 kernel time table (rocprofv3 --kernel-trace --stats) for the per-kernel split of its step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg5s
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfg5s/prof -o run -- python bench_configs.py --config 5 --steps 10 --warmup 3 > gpurun_out/cfg5s/run.log 2>&1 || { tail -5 gpurun_out/cfg5s/run.log; exit 1; }
tail -n 1 gpurun_out/cfg5s/run.log
echo cfg5-stats-done
