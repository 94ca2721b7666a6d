# r03: diag16 microbench + register Cholesky probe + BA parity tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 60 ./tools/ubench/diag16
timeout -k 5 120 python3 tools/probe_cholesky_reg.py 31 100 294 304 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 5 120 python3 tools/probe_cholesky_blocked.py 294 1000 2394 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_ba.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_ba.log; exit $rc
