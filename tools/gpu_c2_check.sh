# Extraction / golden parity on the GPU, then the C2 trace and a short bench (no CPU leg).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_golden.py tests/test_match_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c2_tests.log 2>&1; rc=$?; tail -3 gpurun_out/c2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/trace_c2.py 2>&1 | grep -v amdgpu.ids && \
timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 300 > gpurun_out/bench_c2.log 2>&1; rc=$?; tail -1 gpurun_out/bench_c2.log | cut -c1-200; exit $rc
