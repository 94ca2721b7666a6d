# Blocked / register Cholesky: probe timings + the BA parity tests that run through them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/probe_cholesky_blocked.py 294 1000 2394 > gpurun_out/chol_probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/chol_probe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_K:-} > gpurun_out/ba_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ba_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -u tools/time_gba.py > gpurun_out/time_gba.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/time_gba.log | tail -5; exit $rc
