# r05: T_{k+1} column-k term on wave 1 (A/B against tw0), DAG / ND / BA tests, C4 / C5 times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_tw1
mkdir -p $O
for v in main tw0; do
  if [ $v = main ]; then lib=""; else lib=tools/ubench/ab/liborbhip_$v.so; fi
  ORBHIP_PROBE_LIB=$lib timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 570:loop 2394:loop > $O/probe_$v.log 2>&1 || { tail -20 $O/probe_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/probe_$v.log | grep -v "backward steps"
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ba_gpu.py tests/test_nd_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
ORBHIP_BA_TIMING=1 timeout -k 10 120 python3 -u tools/time_ba.py 20 > $O/time_ba.log 2>&1 || exit 1
tail -2 $O/time_ba.log
ORBHIP_BA_TIMING=1 timeout -k 10 180 python3 -u tools/time_gba.py > $O/time_gba.log 2>&1 || exit 1
tail -2 $O/time_gba.log
timeout -k 10 180 python3 -u tools/time_nd_levels.py 20 > $O/nd_levels.log 2>&1 || exit 1
grep -v amdgpu.ids $O/nd_levels.log
