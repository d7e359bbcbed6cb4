# Round 3: gradient-audit A/B between two library builds (GS_MI355X_LIB) on the audit-printing tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/accab
K="test_stale_partial or test_bench_workload_parity or test_config2_colmap or test_general_camera_full or test_colmap_rotated_poses_full or test_config1_parity"
for L in ${LIBS:-libgs_mi355x.so libgs_chan.so}; do
  GS_MI355X_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -v -s --timeout 300 --timeout-method thread -k "$K" > gpurun_out/accab/$L.log 2>&1
  echo "== $L rc=$?"; grep -E "gradient bar|PASSED|FAILED" gpurun_out/accab/$L.log | cut -c1-330
done
