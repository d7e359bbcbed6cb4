set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab gpurun_out/cfg
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -1 gpurun_out/ab/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/bench_mi355x.log 2>&1 || exit 1
timeout -k 10 400 python bench_configs.py --config 5 > gpurun_out/cfg/cfg5.log 2>&1 || { tail -5 gpurun_out/cfg/cfg5.log; exit 1; }
echo ok
