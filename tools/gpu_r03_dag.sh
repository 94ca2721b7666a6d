# r03: probe the persistent DAG Cholesky (small sizes first; every step time-limited)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 60 python3 -u tools/probe_cholesky_dag.py 31:dense 64:dense 100:dense 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 5 90 python3 -u tools/probe_cholesky_dag.py 294:dense 600:band 1201:dense 2394:loop 2394:dense 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 5 120 python3 -u tools/probe_cholesky_blocked.py 294 1000 2394 2>&1 | grep -v amdgpu.ids
