# GPU box: FETCH_SIZE / WRITE_SIZE passes over a short bench run -> per-kernel HBM bytes per launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tq
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/tq/fetch -o run -- $B > gpurun_out/tq/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/tq/write -o run -- $B > gpurun_out/tq/write.log 2>&1 || exit 1
echo done
