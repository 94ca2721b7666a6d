# r05: LBA latency during a GBA on another context, narrowed hand-off vs r04's tail hand-off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_conc
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ba_concurrent_gpu.py tests/test_ba_gpu.py tests/test_nd_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in after tail after tail; do
  if [ $v = tail ]; then export ORBHIP_DAG_HANDOFF_TAIL=1; else unset ORBHIP_DAG_HANDOFF_TAIL; fi
  timeout -k 10 180 python3 -u tools/time_concurrent.py 2>&1 | grep -v amdgpu || exit 1
done
