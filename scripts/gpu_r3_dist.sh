# Round 3: the N>1 bench line on one GPU (2 ranks over gloo, full 1M size) with its communication
# fields, then a 1-GPU bench and a process listing after it exits (what outlives bench.py?).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3d
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo \
    > gpurun_out/r3d/bench_dist2.log 2>&1 || { tail -20 gpurun_out/r3d/bench_dist2.log; exit 1; }
grep '^{' gpurun_out/r3d/bench_dist2.log > gpurun_out/r3d/bench_dist2.json
python -c "
import json; d=json.load(open('gpurun_out/r3d/bench_dist2.json'))
print({k: d[k] for k in ('value','ms_per_step','comm_gbs')}); print(d['comm']); print(d['stage_ms'])"
ps -eo pid,ppid,user,stat,etime,cmd --forest > gpurun_out/r3d/ps_before.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3d/bench1.json 2> gpurun_out/r3d/bench1.err || exit 1
ps -eo pid,ppid,user,stat,etime,cmd --forest > gpurun_out/r3d/ps_after.txt
sleep 2
ps -eo pid,ppid,user,stat,etime,cmd --forest > gpurun_out/r3d/ps_after2.txt
cut -c1-300 gpurun_out/r3d/bench1.json
