# r05: chain probe, C4 / C5 times, the C5 nested-dissection roofline, BA tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_chain5
mkdir -p $O
timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 570:loop 2394:loop > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
ORBHIP_BA_TIMING=1 timeout -k 10 120 python3 -u tools/time_ba.py 20 > $O/time_ba.log 2>&1 || exit 1
tail -2 $O/time_ba.log
timeout -k 10 180 python3 -u tools/time_gba.py > $O/time_gba.log 2>&1 || exit 1
cat $O/time_gba.log
timeout -k 10 120 python3 -u -c "import bench, json; print(json.dumps(bench.ba_nd_roofline()))" > $O/nd_roofline.log 2>&1 || { tail -5 $O/nd_roofline.log; exit 1; }
cat $O/nd_roofline.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ba_gpu.py tests/test_nd_gpu.py tests/test_ba_concurrent_gpu.py tests/test_ba_sharded_nd_gpu.py > $O/pytest_ba.log 2>&1; rc=$?
tail -3 $O/pytest_ba.log
exit $rc
