# One GPU call for the round's evidence: parity tests, smoke, the bench line (with cpu_baseline),
# the rocprofv3 kernel-trace summary, PMC traffic passes, SQ counters, configs 2 and 5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
[ -n "$SKIP_CHECK" ] || bash scripts/gpu_check.sh || exit 1
bash scripts/gpu_profile_round.sh || exit 1
bash scripts/gpu_sq.sh || exit 1
mkdir -p gpurun_out/cfg
timeout -k 10 300 python bench_configs.py --config 2 > gpurun_out/cfg/cfg2.log 2>&1 || { tail -5 gpurun_out/cfg/cfg2.log; exit 1; }
timeout -k 10 400 python bench_configs.py --config 5 > gpurun_out/cfg/cfg5.log 2>&1 || { tail -5 gpurun_out/cfg/cfg5.log; exit 1; }
# config 5's HBM traffic (one counter group per pass, kernel-trace only)
for c in FETCH_SIZE WRITE_SIZE; do
  d=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/cfg/pmc5/$d -o run -- python bench_configs.py --config 5 --steps 3 --warmup 2 > gpurun_out/cfg/pmc5_$d.log 2>&1 || { tail -5 gpurun_out/cfg/pmc5_$d.log; exit 1; }
done
timeout -k 10 400 python bench_configs.py --config 5 --depth-sort 2 > gpurun_out/cfg/cfg5_d2.log 2>&1 || { tail -5 gpurun_out/cfg/cfg5_d2.log; exit 1; }
timeout -k 10 300 python bench_configs.py --config 2 --depth-sort 2 > gpurun_out/cfg/cfg2_d2.log 2>&1 || { tail -5 gpurun_out/cfg/cfg2_d2.log; exit 1; }
# this user's processes after the runs (none of ours may outlive them)
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > gpurun_out/round/ps_after.txt 2>&1 || true
echo all-done
