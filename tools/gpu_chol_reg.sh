# Register Cholesky: direct solver tests, the probe's phase cycles, then the BA parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k cholesky > gpurun_out/chol_tests.log 2>&1
rc=$?; tail -3 gpurun_out/chol_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -u tools/probe_cholesky_reg.py 96 294 > gpurun_out/chol_reg_probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/chol_reg_probe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ba_tests.log; exit $rc
