# SearchForInitialization parity + timing on the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_init_match.py tests/test_projection.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/init_tests.log 2>&1; rc=$?; tail -14 gpurun_out/init_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/time_init.py 2>&1 | grep -v amdgpu.ids && \
ORBHIP_INIT_CHAIN=1 timeout -k 10 300 python tools/time_init.py 2>&1 | grep -v amdgpu.ids
