# bench_configs.py configs under each depth-sort mode (0 auto, 1 global, 2 per tile): CFGS="2 5" MODES="0 1 2"
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/cfg
for c in ${CFGS:-2 5}; do for d in ${MODES:-0 1 2}; do
  timeout -k 10 300 python bench_configs.py --config $c --depth-sort $d > gpurun_out/cfg/cfg${c}_d${d}.log 2>&1 || { tail -5 gpurun_out/cfg/cfg${c}_d${d}.log; exit 1; }
  python - gpurun_out/cfg/cfg${c}_d${d}.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d.get("stage_ms", {}).items()})
PY
done; done
