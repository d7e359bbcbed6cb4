# Round 3: backward launch positions with the front quarters after every other job: split tests,
# then bench.py --backward-split -1 / 4096 / 2048 / 0
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/split2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for S in -1 4096 2048 0; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --backward-split $S > $O/b_$S.log 2>&1 || { tail -5 $O/b_$S.log; exit 1; }
python -c "import json; d=json.loads(open('$O/b_$S.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('split $S', round(d['ms_per_step'],4), 'bwd', round(s['backward_blend'],4))"
done; done
