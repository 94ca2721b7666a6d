# r05: chain probe + diag16 ubench + C4/C5 times + BA tests on the current tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_chain4
mkdir -p $O
timeout -k 10 60 ./tools/ubench/diag16 > $O/diag16.log 2>&1; echo "diag16 rc=$?"
grep -E "chain|pd,|non-PD" $O/diag16.log
timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 570:loop 2394:loop > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
ORBHIP_BA_TIMING=1 timeout -k 10 120 python3 -u tools/time_ba.py 20 > $O/time_ba.log 2>&1 || exit 1
tail -2 $O/time_ba.log
timeout -k 10 180 python3 -u tools/time_gba.py > $O/time_gba.log 2>&1 || exit 1
cat $O/time_gba.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ba_gpu.py tests/test_nd_gpu.py tests/test_ba_concurrent_gpu.py > $O/pytest_ba.log 2>&1; rc=$?
tail -3 $O/pytest_ba.log
exit $rc
