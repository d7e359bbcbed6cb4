# Rehearse the N>1 bench paths on a single-GPU box: `bench.py --gpus 2` starts its own 2 ranks
# (gaussiansplatting_amd/launch.py), both on cuda:0, gradients reduced over gloo; then config 5's
# full train step at 2 ranks (all-reduce, and the sharded Adam); then the N > 1 step shape on a one-rank
# RCCL group (bench.py --rccl-single-rank: RCCL refuses two ranks on one device).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --gaussians 200000 --dist-backend gloo \
    > gpurun_out/dist/bench_dist2.log 2>&1; rc=$?; tail -2 gpurun_out/dist/bench_dist2.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench_configs.py --config 5 --gpus 2 --steps 3 --warmup 2 --gaussians 500000 \
    --dist-backend gloo > gpurun_out/dist/cfg5_dist2.log 2>&1; rc=$?; tail -2 gpurun_out/dist/cfg5_dist2.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench_configs.py --config 5 --gpus 2 --steps 3 --warmup 2 --gaussians 500000 \
    --dist-backend gloo --sharded-adam > gpurun_out/dist/cfg5_dist2_sharded.log 2>&1; rc=$?; tail -2 gpurun_out/dist/cfg5_dist2_sharded.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --rccl-single-rank --steps 20 --warmup 3 \
    > gpurun_out/dist/bench_rccl1.log 2> gpurun_out/dist/bench_rccl1.err; rc=$?; tail -1 gpurun_out/dist/bench_rccl1.log | cut -c1-400; exit $rc
