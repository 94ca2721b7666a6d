# r05: two-phase k_nd_backsolve; DAG defaults (flag-ahead off, row backward); times + tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_bs
mkdir -p $O
ORBHIP_PREP_DBG=1 timeout -k 10 120 python3 -u tools/time_prep.py > $O/prep.log 2>&1 || { tail -20 $O/prep.log; exit 1; }
grep -v "prepare E=" $O/prep.log; grep "prepare E=80000" $O/prep.log | tail -3
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nd_gpu.py > $O/pytest_nd.log 2>&1 || { tail -30 $O/pytest_nd.log; exit 1; }
tail -2 $O/pytest_nd.log
timeout -k 10 180 python3 -u tools/time_nd_levels.py 20 > $O/nd_levels.log 2>&1 || { tail -20 $O/nd_levels.log; exit 1; }
grep -v amdgpu.ids $O/nd_levels.log
timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 570:loop > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | grep -v sub-phases
ORBHIP_BA_TIMING=1 timeout -k 10 120 python3 -u tools/time_ba.py 20 > $O/time_ba.log 2>&1 || exit 1
tail -2 $O/time_ba.log
for l in 1 2; do ORBHIP_ND_LEVELS=$l ORBHIP_BA_TIMING=1 timeout -k 10 180 python3 -u tools/time_gba.py > $O/time_gba_l$l.log 2>&1 || exit 1; tail -2 $O/time_gba_l$l.log; done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py tests/test_ba_sharded_nd_gpu.py tests/test_ba_concurrent_gpu.py > $O/pytest_ba.log 2>&1; rc=$?
tail -5 $O/pytest_ba.log
exit $rc
