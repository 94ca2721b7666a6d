# r03: state of the tree: full -m gpu suite, smoke, quick bench. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[1/3] pytest -m gpu"
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15; [ $rc -eq 0 ] || exit $rc
echo "[2/3] smoke"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "[3/3] bench"
timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log | tail -1 | cut -c1-3000
