set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_ba_gpu.py -x -q --timeout 120 --timeout-method thread -k "dag or lba_c4" > gpurun_out/r06_probe_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_probe_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 600:band 2394:loop > gpurun_out/r06_probe_dag.log 2>&1 || { tail -5 gpurun_out/r06_probe_dag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_probe_dag.log
timeout -k 10 300 python3 -u -m pytest tests/test_extract_gpu.py tests/test_golden.py tests/test_frontend.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_extract_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_extract_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/ubench/dpp64_check > gpurun_out/r06_dpp64_check.log 2>&1; cat gpurun_out/r06_dpp64_check.log
