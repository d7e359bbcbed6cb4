# Config 5 under each (depth order, tile sort path) pair, with a kernel time table for the per-tile
# order on the one-pass tile sort.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg5p
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_optim.py tests/test_gpu_parity.py -k "adam or packed" > gpurun_out/cfg5p/tests.log 2>&1 || { tail -20 gpurun_out/cfg5p/tests.log; exit 1; }
tail -2 gpurun_out/cfg5p/tests.log
for dt in "2 1" "1 1" "2 2"; do
  set -- $dt
  timeout -k 10 300 python bench_configs.py --config 5 --depth-sort $1 --tile-sort-path $2 > gpurun_out/cfg5p/d$1_t$2.log 2>&1 || { tail -5 gpurun_out/cfg5p/d$1_t$2.log; exit 1; }
  tail -n 1 gpurun_out/cfg5p/d$1_t$2.log | python -c "import json,sys; d=json.load(sys.stdin); print('d$1 t$2', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfg5p/prof -o run -- python bench_configs.py --config 5 --depth-sort 2 --tile-sort-path 1 --steps 5 --warmup 2 > gpurun_out/cfg5p/prof.log 2>&1 || { tail -5 gpurun_out/cfg5p/prof.log; exit 1; }
echo cfg5-paths-done
