# GPU-box A/B over bench.py flag sets (one library): FLAGSETS="name1:--flag a|name2:--flag b", REPS.
# bench lines under gpurun_out/ab/bench_<name>_<rep>.log, summary by ab_summary.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
rm -f $O/bench_*.log $O/cfg*.log
IFS='|' read -ra SETS <<< "${FLAGSETS:-base:}"
for r in $(seq 1 ${REPS:-2}); do
  for s in "${SETS[@]}"; do
    name=${s%%:*}; flags=${s#*:}
    timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline $flags > $O/bench_${name}_$r.log 2>&1 || { tail -5 $O/bench_${name}_$r.log; exit 1; }
  done
done
IFS='|' read -ra CSETS <<< "${CFGSETS:-}"
for s in "${CSETS[@]}"; do
  name=${s%%:*}; flags=${s#*:}
  timeout -k 10 400 python bench_configs.py $flags > $O/cfg_${name}.log 2>&1 || { tail -5 $O/cfg_${name}.log; exit 1; }
done
python scripts/ab_summary.py
echo ab-done
