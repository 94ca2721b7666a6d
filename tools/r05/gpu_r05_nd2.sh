# r05: two-level dissection timing + parity, RCCL local segments, C4 / C5 times, BA tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_nd2
mkdir -p $O
timeout -k 10 180 python3 -u tools/time_nd_levels.py 20 > $O/nd_levels.log 2>&1 || { tail -20 $O/nd_levels.log; exit 1; }
cat $O/nd_levels.log
timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 570:loop > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
tail -12 $O/probe.log
ORBHIP_BA_TIMING=1 timeout -k 10 120 python3 -u tools/time_ba.py 20 > $O/time_ba.log 2>&1 || exit 1
tail -2 $O/time_ba.log
timeout -k 10 180 python3 -u tools/time_gba.py > $O/time_gba.log 2>&1 || exit 1
cat $O/time_gba.log
ORBHIP_ND_LEVELS=1 timeout -k 10 180 python3 -u tools/time_gba.py > $O/time_gba_l1.log 2>&1 || exit 1
cat $O/time_gba_l1.log
for k in 6 8 10; do ORBHIP_ND_K=$k timeout -k 10 180 python3 -u tools/time_gba.py > $O/time_gba_k$k.log 2>&1 || exit 1; tail -1 $O/time_gba_k$k.log; done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_nd_gpu.py tests/test_ba_sharded_nd_gpu.py tests/test_ba_sharded_gpu.py tests/test_ba_gpu.py tests/test_ba_concurrent_gpu.py > $O/pytest_ba.log 2>&1; rc=$?
tail -5 $O/pytest_ba.log
exit $rc
