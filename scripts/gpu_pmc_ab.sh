# A/B of library variants with the -m gpu suite on the first, bench reps, and one FETCH/WRITE PMC
# pass pair per variant summarised by pmc_traffic.py (per-kernel read/write MB per launch).
#   VARIANTS="mi355x foo" REPS=2 bash scripts/gpu_pmc_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pab; mkdir -p $O
first=${VARIANTS%% *}
if [ -z "$NOTESTS" ]; then
  GS_MI355X_LIB=libgs_$first.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "== tests $first: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -30 $O/pytest.log; exit $rc; }
fi
for v in $VARIANTS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    GS_MI355X_LIB=libgs_$v.so timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$v/$d -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 3 $BENCH_ARGS > $O/pmc_${v}_$d.log 2>&1 || { tail -5 $O/pmc_${v}_$d.log; exit 1; }
    f=$(find $O/pmc_$v/$d -name run_counter_collection.csv | head -1); [ -f $O/pmc_$v/$d/run_counter_collection.csv ] || cp $f $O/pmc_$v/$d/
  done
  python scripts/pmc_traffic.py $O/pmc_$v ab_$v 1000000 4651618 1920 1080 > $O/traffic_$v.txt 2>&1 || true
  echo "== traffic $v"; cat $O/traffic_$v.txt
done
REPS=${REPS:-3} VARIANTS="$VARIANTS" CFG=$CFG PROF=$PROF bash scripts/ab.sh
