# r05: the whole -m gpu suite and smoke on the current tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_suite
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
