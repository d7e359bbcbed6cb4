# Rehearse the N>1 bench path on a single-GPU box: 2 ranks share cuda:0, gradients reduced over gloo.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --gaussians 200000 --dist-backend gloo \
    > gpurun_out/bench_dist2.log 2>&1; rc=$?; tail -3 gpurun_out/bench_dist2.log | cut -c1-400; exit $rc
