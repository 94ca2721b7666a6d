# r05: the whole -m gpu suite and smoke on the current tree (no bench)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r05_pytest_gpu_mid.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r05_pytest_gpu_mid.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|ERROR" gpurun_out/r05_pytest_gpu_mid.log | head; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_mid.log 2>&1 || { tail -5 gpurun_out/r05_smoke_mid.log; exit 1; }
tail -1 gpurun_out/r05_smoke_mid.log
