# BA pipeline check: parity tests (LBA/GBA/sharded), C4 single + batched timing, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py tests/test_pose_opt.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; tail -15 gpurun_out/ba_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -u tools/time_ba.py 20 256 > gpurun_out/time_ba.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/time_ba.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ba -o run -- python3 tools/time_ba.py 5 256 > gpurun_out/prof_ba.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
