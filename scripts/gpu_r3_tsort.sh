# Config 5 (bench_configs.py) per tile-sort path: bash scripts/gpu_r3_tsort.sh "0 1 2 3"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ts
for path in ${1:-0 1 2 3}; do
  timeout -k 10 300 python bench_configs.py --config 5 --tile-sort-path $path > gpurun_out/ts/cfg5_$path.log 2>&1 || { tail -5 gpurun_out/ts/cfg5_$path.log; exit 1; }
  python - <<PY
import json
d = json.loads([l for l in open('gpurun_out/ts/cfg5_$path.log') if l.startswith('{')][-1])
print('path $path', round(d['ms_per_step'], 4), ' '.join(f'{k}={v:.4f}' for k, v in d.get('stage_ms', {}).items()), d.get('config', {}).get('pairs_per_view'))
PY
done
