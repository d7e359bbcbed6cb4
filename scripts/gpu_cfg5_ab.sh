set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg5ab
for v in mi355x old; do
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 400 python bench_configs.py --config 5 > gpurun_out/cfg5ab/$v.log 2>&1 || { tail -5 gpurun_out/cfg5ab/$v.log; exit 1; }
  echo "$v $(tail -n 1 gpurun_out/cfg5ab/$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), {k: round(v,3) for k,v in d.get("stage_ms",{}).items()})')"
done
GS_MI355X_LIB=libgs_old.so timeout -k 10 400 python bench_configs.py --config 5 > /dev/null 2>&1 || true
