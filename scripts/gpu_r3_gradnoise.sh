# Round 3 diagnostics: which float step of the backward moves the deep-list gradient entries
# (hardware exp, rcp instead of IEEE division, fused acc/dd) -- the audit of each variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3n
for v in mi355x pexp idiv refacc allref; do
  GS_MI355X_LIB=libgs_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -m gpu -v -s --timeout 250 --timeout-method thread \
    -k "general_camera_full or bench_workload" > gpurun_out/r3n/$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; grep -E "^gradient bar|^tests.*gradient bar" gpurun_out/r3n/$v.log | sed 's/widened_per_field.*//'
  [ $rc -le 1 ] || exit 1
done
