# GPU-box: one rocprofv3 SQ-counter pass over a short bench run (instruction mix / stall analysis).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline"
C=${SQ_COUNTERS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"}
timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/sq -o run -- $B > gpurun_out/sq/sq.log 2>&1 || exit $?
C2=${SQ_COUNTERS2:-"SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"}
timeout -k 10 400 rocprofv3 --pmc $C2 --kernel-trace --output-format csv -d gpurun_out/sq2 -o run -- $B > gpurun_out/sq/sq2.log 2>&1 || exit $?
echo done
