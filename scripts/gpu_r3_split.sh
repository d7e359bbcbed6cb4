# Round 3: backward list split -- parity, bench A/B over the split count, tail traces.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 240 --timeout-method thread \
    -k "split or stale or graph_replay or bench_workload or config1 or packed or deterministic or general_camera" > gpurun_out/r3s/tests.log 2>&1 \
    || { grep -E "PASSED|FAILED|^E " gpurun_out/r3s/tests.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/r3s/tests.log | tail -2
for s in 0 -1 4096 2048 0 -1; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --backward-split $s > gpurun_out/r3s/bench_$s.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/r3s/bench_$s.json')); st=d['stage_ms']
print('split $s', round(d['ms_per_step'],4), 'bwd', round(st['backward_blend'],4), 'chain', round(st['chain'],4), 'fwd', round(st['forward_blend'],4))"
done
for s in 0 -1; do
  GS_MI355X_LIB=libgs_btrace.so timeout -k 10 200 python scripts/blend_trace2.py $s > gpurun_out/r3s/trace_$s.txt 2>&1 || { tail -5 gpurun_out/r3s/trace_$s.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r3s/trace_$s.txt
done
