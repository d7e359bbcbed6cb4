# Round 3: chain kernel choice -- parity (incl. both chain kernels), bench, config 5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/chain2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_train_sequence.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print('bench', round(d['ms_per_step'],4), 'chain', round(d['stage_ms']['chain'],4))"
timeout -k 10 400 python bench_configs.py --config 5 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/c5.log').read().strip().splitlines()[-1]); print('cfg5', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items()})"
done
