# Projection searches + extraction parity on the GPU, timing of the searches and a short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_projection.py tests/test_extract_gpu.py -x -q -m gpu > gpurun_out/proj_tests.log 2>&1; rc=$?; tail -4 gpurun_out/proj_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/time_proj.py 2>&1 | grep -v amdgpu.ids && \
timeout -k 10 300 python bench.py --no-cpu --steps 300 > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-300; grep -o '"c3_1280x720[^,]*' gpurun_out/bench.log; exit $rc
