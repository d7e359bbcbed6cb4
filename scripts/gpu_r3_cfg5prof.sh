# Round 3: kernel-trace stats of bench_configs config 5 (tile-sort path $TSP)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/cfg5prof; mkdir -p $O
for p in ${TSPS:-3 2}; do
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$p -o c -- python bench_configs.py --config 5 --tile-sort-path $p > $O/p$p.log 2>&1 || exit 1
python - $O/p$p/c_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-45s calls %6s avg %9.1f us" % (r['Name'].split('(')[0][:45], r['Calls'], float(r['AverageNs'])/1e3))
PY
done
