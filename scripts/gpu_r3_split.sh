# Round 3: how many tiles split their backward (bench.py --backward-split; default -1 = all) with the
# XCD-group launch order: alternating bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/split; mkdir -p $O
for i in 1 2 3; do for S in -1 4096 2048; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --backward-split $S > $O/b_$S.log 2>&1 || { tail -5 $O/b_$S.log; exit 1; }
python -c "import json; d=json.loads(open('$O/b_$S.log').read().strip().splitlines()[-1]); s=d['stage_ms']; print('split $S', round(d['ms_per_step'],4), 'bwd', round(s['backward_blend'],4))"
done; done
