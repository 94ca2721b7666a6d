# r06 (late): the BA suites on the current tree, the C4 / C5 timings through the C-ABI, and the
# chain probe at n = 294 (debug build's interval and backward-step cycles)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r06/gpu_batests.sh || exit 1
timeout -k 10 60 python3 tools/probe_cholesky_dag.py 294:dense 600:band > gpurun_out/r06_probe_dag.log 2>&1 || { tail -5 gpurun_out/r06_probe_dag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_probe_dag.log
