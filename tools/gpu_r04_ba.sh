# r04: the BA / projection GPU tests (concurrent contexts, forced DAG timeout, parity), one process
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_ba_concurrent_gpu.py tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py tests/test_projection.py} \
    -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r04_ba.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r04_ba.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|ERROR|Error" gpurun_out/r04_ba.log | head -20; exit $rc; }
