# r05: the DPP diagonal factorization (diag16_cl / diag16_dpp) in isolation and inside the
# persistent Cholesky (A/B against the r04 pivot-block form), plus the BA parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_chain
mkdir -p $O
timeout -k 10 60 ./tools/ubench/diag16 > $O/diag16.log 2>&1; echo "diag16 rc=$?"
grep -E "chain|pd,|non-PD" $O/diag16.log
export ORBHIP_PROBE_SAVE=$O
timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 912:loop 2394:loop > $O/probe_new.log 2>&1 || { tail -20 $O/probe_new.log; exit 1; }
cat $O/probe_new.log
ORBHIP_PROBE_LIB=tools/ubench/ab/liborbhip_olddiag.so timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 912:loop 2394:loop > $O/probe_old.log 2>&1 || { tail -20 $O/probe_old.log; exit 1; }
cat $O/probe_old.log
timeout -k 10 120 python3 -u tools/time_ba.py 20 > $O/time_ba.log 2>&1 || exit 1
cat $O/time_ba.log
timeout -k 10 180 python3 -u tools/time_gba.py > $O/time_gba.log 2>&1 || exit 1
cat $O/time_gba.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ba_gpu.py tests/test_nd_gpu.py tests/test_ba_concurrent_gpu.py > $O/pytest_ba.log 2>&1; rc=$?
tail -5 $O/pytest_ba.log
exit $rc
