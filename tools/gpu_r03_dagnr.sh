# r03: DAG probe with 1 (default build) and 2 Newton steps (separate test library build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 5 90 python3 -u tools/probe_cholesky_dag.py 64:dense 294:dense 2394:loop 2394:dense 2>&1 | grep -v amdgpu.ids || exit 1
echo "--- 2 Newton steps"
ORBHIP_PROBE_LIB=tools/ubench/liborbhip_nr2.so timeout -k 5 90 python3 -u tools/probe_cholesky_dag.py 294:dense 2394:loop 2>&1 | grep -v amdgpu.ids
