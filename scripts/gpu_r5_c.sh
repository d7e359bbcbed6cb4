# The new defaults (in-forward per-tile sort, depth-sort jobs): the -m gpu suite, the bench line,
# configs 2 and 5 under both depth orders.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== tests"; SHOW=4 bash scripts/gpu_tests.sh || exit $?
mkdir -p gpurun_out/cfg
echo "== bench"; timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c.log 2>&1 || { tail -5 gpurun_out/bench_c.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_c.log').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()})"
for a in "2 0" "2 2" "5 0" "5 2"; do set -- $a
  timeout -k 10 400 python bench_configs.py --config $1 --depth-sort $2 > gpurun_out/cfg/cfg$1_d$2.log 2>&1 || { tail -5 gpurun_out/cfg/cfg$1_d$2.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/cfg/cfg$1_d$2.log').read().strip().splitlines()[-1]); print('cfg$1 d$2', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()})"
done
