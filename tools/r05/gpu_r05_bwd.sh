# r05: column-form backward + flag-ahead A/B (probe), DAG / BA / shard tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_bwd
mkdir -p $O
for v in main fa0 bk0; do
  if [ $v = main ]; then lib=""; else lib=tools/ubench/ab/liborbhip_$v.so; fi
  ORBHIP_PROBE_LIB=$lib timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 570:loop 2394:loop > $O/probe_$v.log 2>&1 || { tail -20 $O/probe_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/probe_$v.log
done
ORBHIP_BA_TIMING=1 timeout -k 10 120 python3 -u tools/time_ba.py 20 > $O/time_ba.log 2>&1 || exit 1
tail -2 $O/time_ba.log
timeout -k 10 180 python3 -u tools/time_gba.py > $O/time_gba.log 2>&1 || exit 1
tail -1 $O/time_gba.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py tests/test_ba_sharded_nd_gpu.py tests/test_nd_gpu.py tests/test_ba_concurrent_gpu.py > $O/pytest_ba.log 2>&1; rc=$?
tail -5 $O/pytest_ba.log
exit $rc
