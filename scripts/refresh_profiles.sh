# Copy the evidence of scripts/gpu_round_a.sh + gpu_round_b.sh (merged back into gpurun_out/) into profiles/:
# bench line, rocprofv3 kernel stats, PMC traffic (traffic.json), SQ counters (valu.json), configs 2/5.
set -e
cd "$(dirname "$0")/.."
W=1000000g_1920x1080
R=${ROUND_TAG:-r06}
# every input must be there before any profile is overwritten
for f in gpurun_out/round/bench.log gpurun_out/round/prof/bench_kernel_stats.csv gpurun_out/sq/run_counter_collection.csv \
         gpurun_out/sq2/run_counter_collection.csv gpurun_out/cfg/cfg2.log gpurun_out/cfg/cfg5.log; do
  [ -s "$f" ] || { echo "missing $f: run scripts/gpu_round_a.sh and gpu_round_b.sh first" >&2; exit 1; }
done
tail -n 1 gpurun_out/round/bench.log > profiles/${R}_bench.json
cp gpurun_out/round/prof/bench_kernel_stats.csv profiles/${R}_kernel_stats.csv
P=$(python -c "import json; print(json.loads(open('gpurun_out/round/bench.log').read().strip().splitlines()[-1])['config']['pairs_per_view'])")
{ echo "# HBM bytes per launch (rocprofv3 PMC: 2 x FETCH_SIZE + WRITE_SIZE, KiB x 1024) against each kernel's"
  echo "# algorithmic bytes per launch; bench workload 1M Gaussians 1080p, P = $P"
  python scripts/pmc_traffic.py gpurun_out/round/pmc $W 1000000 $P 1920 1080 gpurun_out/round/prof/bench_kernel_stats.csv \
      --facts gpurun_out/round/bench.log; } > profiles/${R}_pmc_traffic.txt
if [ -s gpurun_out/cfg/pmc5/fetch/run_counter_collection.csv ]; then
  J5=$(tail -n 1 gpurun_out/cfg/cfg5.log)
  N5=$(echo "$J5" | python -c "import json,sys; print(json.load(sys.stdin)['config']['gaussians'])")
  P5=$(echo "$J5" | python -c "import json,sys; print(json.load(sys.stdin)['config']['pairs_per_view'])")
  { echo "# config 5 (full train step after the density apply): N = $N5, P = $P5; per-launch means over every"
    echo "# launch of the run: kernels that only run in the warm-up frames before the apply (5M Gaussians, the"
    echo "# first frame on the per-tile order) are set against the 5.2M-Gaussian sizes"
    python scripts/pmc_traffic.py gpurun_out/cfg/pmc5 cfg5_${N5}g_1920x1080 $N5 $P5 1920 1080 \
        --facts gpurun_out/cfg/cfg5.log; } > profiles/${R}_pmc_traffic_cfg5.txt
fi
python scripts/sq_valu.py gpurun_out/sq/run_counter_collection.csv $W > /dev/null
{ echo "# issue efficiency (fractions of SQ_WAVE_CYCLES; scripts/sq_issue.py)"
  python scripts/sq_issue.py gpurun_out/sq/run_counter_collection.csv gpurun_out/sq2/run_counter_collection.csv
  echo; echo "# per-kernel counter means per dispatch (scripts/sq_summary.py)"
  python scripts/sq_summary.py gpurun_out/sq/run_counter_collection.csv gpurun_out/sq2/run_counter_collection.csv; } > profiles/${R}_sq_counters.txt
[ -s gpurun_out/pytest_gpu.log ] && cp gpurun_out/pytest_gpu.log profiles/${R}_gpu_tests.log
[ -s gpurun_out/round/ps_after.txt ] && cp gpurun_out/round/ps_after.txt profiles/${R}_ps_after_bench.txt
for c in 2 5; do tail -n 1 gpurun_out/cfg/cfg$c.log > profiles/${R}_bench_cfg$c.json; done
# the N > 1 paths rehearsed on the one-GPU box (two gloo ranks on cuda:0, scripts/gpu_dist_rehearsal.sh)
if [ -s gpurun_out/dist/bench_dist2.log ]; then
  tail -n 1 gpurun_out/dist/bench_dist2.log > profiles/${R}_bench_gpus2_gloo.json
  tail -n 1 gpurun_out/dist/cfg5_dist2.log > profiles/${R}_bench_cfg5_gpus2_gloo.json
  tail -n 1 gpurun_out/dist/cfg5_dist2_sharded.log > profiles/${R}_bench_cfg5_gpus2_gloo_sharded.json
  [ -s gpurun_out/dist/bench_rccl1.log ] && tail -n 1 gpurun_out/dist/bench_rccl1.log > profiles/${R}_bench_rccl_single_rank.json
fi
R=$R python - <<'EOF'
import csv, json, os
R = os.environ["R"]
b = json.load(open(f"profiles/{R}_bench.json"))
print("bench ms/step %.4f  value %.3e  backward %.4f ms  forward %.4f ms" % (
    b["ms_per_step"], b["value"], b["stage_ms"]["backward_blend"], b["stage_ms"]["forward_blend"]))
for r in csv.DictReader(open(f"profiles/{R}_kernel_stats.csv")):
    n = r["Name"].split("(")[0]
    if "backward_kernel" in n or "forward_kernel" in n or "forward_quad_kernel" in n:
        print("rocprof %-32s avg %.1f us" % (n, float(r["AverageNs"]) / 1e3))
EOF
