# r03: DAG Cholesky probe, BA parity tests (DAG path), single LBA / GBA timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 90 python3 -u tools/probe_cholesky_dag.py 64:dense 294:dense 600:band 2394:loop 2394:dense 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_ba.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_ba.log; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 python3 -u tools/time_ba.py 20 0 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 5 120 python3 -u tools/time_gba.py 400 20000 10 2>&1 | grep -v amdgpu.ids || exit 1
ORBHIP_CHOL_BLOCKED=1 timeout -k 5 120 python3 -u tools/time_gba.py 400 20000 10 2>&1 | grep -v amdgpu.ids
