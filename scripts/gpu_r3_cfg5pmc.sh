# Round 3: config 5 per-kernel HBM traffic and SQ counters (bench_configs --config 5, 3 steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c5pmc; mkdir -p $O
B="python bench_configs.py --config 5 --steps 3 --warmup 1"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- $B > $O/f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- $B > $O/w.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/sq -o run -- $B > $O/s.log 2>&1 || exit 1
python scripts/sq_summary.py $O/sq/run_counter_collection.csv | grep -A1 "offsets_scan\|emit_slots\|project_kernel\|onesweep\|radix\|chain_kernel\|adam"
echo done
