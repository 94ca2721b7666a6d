# k_fast_cells change check: extraction parity, C3 kernel stats (rocprofv3), C2 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_golden.py tests/test_frontend.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fast_tests.log 2>&1; rc=$?; tail -2 gpurun_out/fast_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3ab -o run -- python3 tools/run_c3.py 30 > gpurun_out/prof_c3ab.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --no-extra > gpurun_out/bench_c2ab.log 2>&1
rc=$?; echo rc=$rc; exit $rc
