# A/B of library variants on config 5 (bench_configs.py): bash scripts/gpu_r3_ab5.sh "lib1 lib2 ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab5
for v in $1; do
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 python bench_configs.py --config 5 > gpurun_out/ab5/cfg5_$v.log 2>&1 || { tail -5 gpurun_out/ab5/cfg5_$v.log; exit 1; }
  python - <<PY
import json
line = [l for l in open('gpurun_out/ab5/cfg5_$v.log') if l.startswith('{')][-1]
d = json.loads(line)
print('$v', round(d['ms_per_step'], 4), ' '.join(f'{k}={v:.4f}' for k, v in d.get('stage_ms', {}).items()))
PY
done
