# Pose-only optimizer (and the BA tests sharing ba_se3.h) on the GPU + latency/throughput timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_pose_opt.py tests/test_ba_gpu.py -x -q -m gpu > gpurun_out/pose_tests.log 2>&1; rc=$?; tail -4 gpurun_out/pose_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/time_pose.py 1024 600 2>&1 | grep -v amdgpu.ids
