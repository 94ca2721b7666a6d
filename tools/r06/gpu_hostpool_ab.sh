# r06 (late): C5 / C4 host costs with the host pool on one large problem (default) against the
# calling thread alone (ORBHIP_HOST_POOL=0), alternating runs; ORBHIP_BA_TIMING splits the call
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 0 1 0 1; do
  ORBHIP_HOST_POOL=$m ORBHIP_BA_TIMING=1 timeout -k 10 120 python3 tools/time_gba.py > gpurun_out/hp_$m.log 2>&1 || { tail -5 gpurun_out/hp_$m.log; exit 1; }
  echo "pool=$m $(grep GBA gpurun_out/hp_$m.log)"
  grep "ba timing" gpurun_out/hp_$m.log | tail -2
done
ORBHIP_BA_TIMING=1 timeout -k 10 60 python3 tools/time_ba.py 50 > gpurun_out/hp_c4.log 2>&1 || { tail -5 gpurun_out/hp_c4.log; exit 1; }
grep LBA gpurun_out/hp_c4.log; grep "ba timing" gpurun_out/hp_c4.log | tail -2
timeout -k 10 300 python3 -u -m pytest tests/test_ba_gpu.py tests/test_nd_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/hp_tests.log 2>&1 || { tail -5 gpurun_out/hp_tests.log; exit 1; }
tail -1 gpurun_out/hp_tests.log
