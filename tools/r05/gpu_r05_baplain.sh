# r05: plain stores of the trial's errors (the small problems' refresh moved into k_ba_lin) against
# HEAD (prevba): BA tests, then C4 LBA and C5 GBA timing, alternating runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_baplain
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py tests/test_ba_sharded_nd_gpu.py tests/test_nd_gpu.py tests/test_ba_concurrent_gpu.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in main prevba; do
    unset ORBHIP_LIB
    [ $v = main ] || export ORBHIP_LIB=tools/ubench/ab/liborbhip_$v.so
    echo "$v $(timeout -k 10 120 python3 -u tools/time_ba.py 40 2>/dev/null | tail -1)" || exit 1
    echo "$v $(timeout -k 10 200 python3 -u tools/time_gba.py 2>/dev/null | tail -1)" || exit 1
  done
done
