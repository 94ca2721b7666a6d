# Extraction parity + C3 timing + C2 trace after FAST changes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_golden.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fast_tests.log 2>&1; rc=$?; tail -2 gpurun_out/fast_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/trace_c2.py 2>&1 | grep -A1 k_fast && \
timeout -k 10 200 python tools/trace_c2.py --c3 2>&1 | grep -v amdgpu.ids | head -8
