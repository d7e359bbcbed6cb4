# config 5 with a forced tile-sort path over library variants: bash scripts/gpu_r3_ab5p.sh PATH "lib1 lib2"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab5
for v in $2; do
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 python bench_configs.py --config 5 --tile-sort-path $1 > gpurun_out/ab5/cfg5_$v.log 2>&1 || { tail -5 gpurun_out/ab5/cfg5_$v.log; exit 1; }
  python - <<PY
import json
d = json.loads([l for l in open('gpurun_out/ab5/cfg5_$v.log') if l.startswith('{')][-1])
print('$v', round(d['ms_per_step'], 4), ' '.join(f'{k}={v:.4f}' for k, v in d.get('stage_ms', {}).items()))
PY
done
