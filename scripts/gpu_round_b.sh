# Second half of the round's evidence (after scripts/gpu_round_a.sh: the check and profile steps):
# SQ counters, configs 2 and 5, config 5's PMC traffic passes, the two-rank gloo rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_sq.sh || exit 1
mkdir -p gpurun_out/cfg gpurun_out/round
timeout -k 10 300 python bench_configs.py --config 2 > gpurun_out/cfg/cfg2.log 2>&1 || { tail -5 gpurun_out/cfg/cfg2.log; exit 1; }
timeout -k 10 400 python bench_configs.py --config 5 > gpurun_out/cfg/cfg5.log 2>&1 || { tail -5 gpurun_out/cfg/cfg5.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  d=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/cfg/pmc5/$d -o run -- python bench_configs.py --config 5 --steps 3 --warmup 2 > gpurun_out/cfg/pmc5_$d.log 2>&1 || { tail -5 gpurun_out/cfg/pmc5_$d.log; exit 1; }
done
bash scripts/gpu_dist_rehearsal.sh || exit 1
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > gpurun_out/round/ps_after.txt 2>&1 || true
for f in cfg2 cfg5; do python -c "import json; d=json.loads(open('gpurun_out/cfg/$f.log').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],4))"; done
echo round-b-done
