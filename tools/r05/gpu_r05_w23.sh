# r05: waves 2/3 MFMA chains interleaved (ORBHIP_DAG_W23_EARLY) against the sequential order (w23old):
# BA tests on the new build, then the chain probe and C4 / C5 timing, alternating runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_w23
mkdir -p $O
timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 570:loop > $O/probe_main0.log 2>&1 || { tail -20 $O/probe_main0.log; exit 1; }
cat $O/probe_main0.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ba_gpu.py tests/test_nd_gpu.py tests/test_ba_concurrent_gpu.py tests/test_ba_sharded_nd_gpu.py > $O/pytest_ba.log 2>&1 || { tail -30 $O/pytest_ba.log; exit 1; }
tail -1 $O/pytest_ba.log
for i in 1 2 3; do
  for v in main w23old; do
    unset ORBHIP_LIB ORBHIP_PROBE_LIB
    [ $v = main ] || export ORBHIP_LIB=tools/ubench/ab/liborbhip_$v.so ORBHIP_PROBE_LIB=tools/ubench/ab/liborbhip_$v.so
    timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 570:loop > $O/probe_${v}_$i.log 2>&1 || exit 1
    echo "$v probe: $(grep -E 'us' $O/probe_${v}_$i.log | head -2 | tr '\n' ' ')"
    echo "$v $(timeout -k 10 120 python3 -u tools/time_ba.py 40 2>/dev/null | tail -1)" || exit 1
    echo "$v $(timeout -k 10 200 python3 -u tools/time_gba.py 2>/dev/null | tail -1)" || exit 1
  done
done
