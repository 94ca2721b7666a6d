# r02 final: GPU suite + smoke, default bench line, rocprofv3 kernel stats of the bench (no CPU
# leg), then the PMC passes of every regime (tools/gpu_pmc.sh). Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[1/4] pytest -m gpu"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
echo "[2/4] bench"
timeout -k 10 500 python3 -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log | tail -1 | cut -c1-400
echo "[3/4] rocprofv3 kernel stats"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
echo "[4/4] PMC passes"
bash tools/gpu_pmc.sh
