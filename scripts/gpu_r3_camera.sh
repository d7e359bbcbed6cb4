# Round 3: general-camera parity + the shadow-bar audit (progress on stdout via -s).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 240 --timeout-method thread \
    -k "general_camera or colmap_rotated or config1 or edge_cases or rig_camera" > gpurun_out/r3/small.log 2>&1 || { tail -40 gpurun_out/r3/small.log; exit 1; }
tail -3 gpurun_out/r3/small.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -m gpu -v -s --timeout 600 --timeout-method thread \
    -k "general_camera_full or colmap_rotated_poses_full or config2 or bench_workload" > gpurun_out/r3/full.log 2>&1 || { grep -E "gradient bar|PASS|FAIL|Error|error" gpurun_out/r3/full.log | tail -40; exit 1; }
grep -E "gradient bar|passed|failed" gpurun_out/r3/full.log | tail -20
