# r06: the chain's new backward (column-major copies, no barrier per step): DAG solver tests, the
# BA parity tests, the probe's cycle breakdown, then a quick bench of C4/C5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_ba_gpu.py tests/test_nd_gpu.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r06_bwd_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r06_bwd_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py > gpurun_out/r06_probe_dag.log 2>&1 || { tail -5 gpurun_out/r06_probe_dag.log; exit 1; }
head -12 gpurun_out/r06_probe_dag.log
timeout -k 10 200 python3 -u tools/time_gba.py > gpurun_out/r06_time_gba.log 2>&1 || { tail -5 gpurun_out/r06_time_gba.log; exit 1; }
tail -5 gpurun_out/r06_time_gba.log
