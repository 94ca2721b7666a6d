set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_ba_gpu.py tests/test_nd_gpu.py tests/test_ba_sharded_gpu.py tests/test_ba_sharded_nd_gpu.py tests/test_ba_concurrent_gpu.py tests/test_pose_opt.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_batests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_batests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r06_batests.log | head; exit $rc; }
timeout -k 10 120 python3 tools/time_gba.py 2>&1 | grep GBA
timeout -k 10 60 python3 tools/time_ba.py 50 2>&1 | grep LBA
