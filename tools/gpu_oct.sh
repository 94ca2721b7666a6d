# Octree check: the GPU suite (or PYTEST_FILES), then the C2 device trace (per-phase cycles of level 0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ext_tests.log 2>&1
rc=$?; tail -15 gpurun_out/ext_tests.log; [ $rc -ne 0 ] && exit $rc
ORBHIP_TRACE_BLOCK=0 timeout -k 10 120 python3 -u tools/trace_c2.py > gpurun_out/trace_c2.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/trace_c2.log; exit $rc
