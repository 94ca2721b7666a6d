# Blocked Cholesky: direct solver tests, GBA parity (blocked sizes, C5 full size, shards), probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cb_tests.log 2>&1
rc=$?; tail -4 gpurun_out/cb_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -u tools/probe_cholesky_blocked.py 2>&1 | grep -v amdgpu.ids | tail -8
timeout -k 10 200 python3 -u tools/time_gba.py 2>&1 | grep -v amdgpu.ids | tail -4
