# A/B of library variants on the bench: bash scripts/gpu_r3_ab.sh "lib1 lib2 ..." [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
LIBS="$1"; shift
for rep in 1 2; do
for v in $LIBS; do
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/ab/bench_$v.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/ab/bench_$v.json')); st=d['stage_ms']
print('$v', round(d['ms_per_step'],4), ' '.join(f'{k}={v:.4f}' for k,v in st.items()))"
done
done
