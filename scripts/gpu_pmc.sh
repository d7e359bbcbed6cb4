# GPU-box PMC collection for the roofline `traffic` field (MI355X_MICROARCH.md "HBM"): one
# counter group per rocprofv3 pass, kernel-trace only (no sys/runtime traces with --pmc).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline"
echo "== list"; timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
echo "== fetch"; timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/pmc/fetch -o run -- $B > gpurun_out/pmc/fetch.log 2>&1 || exit $?
echo "== write"; timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats --output-format csv -d gpurun_out/pmc/write -o run -- $B > gpurun_out/pmc/write.log 2>&1 || exit $?
echo "== sq"; timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmc/sq -o run -- $B > gpurun_out/pmc/sq.log 2>&1 || exit $?
echo done
